#!/bin/bash
# Network-side inference: model/sigma tests, then kernel stats of config-2
# fp16 inference through AVRModel.
set -u
OUT=gpurun_out/infer
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_sigma.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -2 $OUT/prof.log
python - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/infer/prof/run_kernel_stats.csv')))[:10]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
