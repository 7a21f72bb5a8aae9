#!/bin/bash
# Graph-replay vs eager throughput in the driver's bench command, 4 runs.
set -u
OUT=gpurun_out/eg
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  tail -1 $OUT/b$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager', round(d['ms_per_step'],4), 'graph', round(d['ms_per_step_graph'],4), 'serial', round(d['ir_render_ms_per_pose'],4))"
done
