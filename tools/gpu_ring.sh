#!/bin/bash
# The driver's bench command with graph rings of 3, 6 and 12 instances per
# stream, 2 and 3 streams, interleaved (value = graph replays; eager beside).
set -u
OUT=gpurun_out/ring
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for cfg in "2 3" "2 6" "2 12" "3 6"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline --streams $1 --graph-ring $2 > $OUT/s$1r$2.$i.log 2>&1 || { tail -20 $OUT/s$1r$2.$i.log; exit 1; }
    tail -1 $OUT/s$1r$2.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams $1 ring $2', round(d['value']/1e9,4), round(d['ms_per_step'],4), round(d['ms_per_step_eager'],4), round(d['host_issue_ms_per_step'],4))"
  done
done
