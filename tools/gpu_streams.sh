#!/bin/bash
# The driver's bench command with 2, 3 and 4 pipelining streams, interleaved.
set -u
OUT=gpurun_out/streams
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for s in 2 3 4; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline --streams $s > $OUT/s$s.$i.log 2>&1 || { tail -20 $OUT/s$s.$i.log; exit 1; }
    tail -1 $OUT/s$s.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams $s', d['value'], d['ms_per_step'], d['ms_per_step_eager'])"
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --no-network --no-cpu-baseline --streams 2 > $OUT/long2.log 2>&1 && tail -1 $OUT/long2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams 2 K=200', d['value'], d['ms_per_step'], d['ms_per_step_eager'])"
