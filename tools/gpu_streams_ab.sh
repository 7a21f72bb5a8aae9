#!/bin/bash
# Pipelined throughput of the driver's bench line at 1, 2, 3 and 4 HIP
# streams, interleaved (--no-network --no-cpu-baseline).
set -u
OUT=gpurun_out/streams_ab
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for s in 2 3 4; do
    timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-network --no-cpu-baseline --streams $s > $OUT/s$s.$i.log 2>&1 || { tail -20 $OUT/s$s.$i.log; exit 1; }
    tail -1 $OUT/s$s.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams', $s, 'run', $i, round(d['ms_per_step'],4), round(d['ms_per_step_graph'],4), round(d['ir_render_ms_per_pose'],4))"
  done
done
