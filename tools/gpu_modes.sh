#!/bin/bash
# The other bench modes at N = 1 (config 5 ray shard, config 4 DDP training),
# each with its CPU leg, plus the 2-rank rehearsal of the launcher.
set -u
OUT=gpurun_out/modes
mkdir -p $OUT
export TMPDIR=/tmp
for m in ray-shard ddp-train; do
  timeout -k 10 400 python bench.py --mode $m --steps 10 --warmup 3 > $OUT/$m.log 2>&1 || { tail -20 $OUT/$m.log; exit 1; }
  tail -1 $OUT/$m.log > $OUT/$m.json
  python -c "import json; d=json.load(open('$OUT/$m.json')); print('$m', d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
done
