#!/bin/bash
# HIP hidden-layer GEMM in situ: model tests, then config-2 fp16 inference
# with it (AVR_LINEAR=1) and with hipBLASLt (0), kernel stats of each.
set -u
OUT=gpurun_out/linear
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_model.py tests/test_gpu_sigma.py tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $OUT/tests2.log 2>&1 || { tail -30 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
for d in 0 1 2 3; do
  AVR_LINEAR_DBG=$d timeout -k 10 200 python tools/probe_linear.py --dtype fp16 > $OUT/dbg$d.log 2>&1 || { tail -20 $OUT/dbg$d.log; exit 1; }
  echo "dbg $d: $(grep avr_linear $OUT/dbg$d.log)"
done
for v in 1 0; do
  AVR_LINEAR=$v timeout -k 10 300 python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 20 --warmup 5 > $OUT/infer$v.log 2>&1 || { tail -20 $OUT/infer$v.log; exit 1; }
  echo "AVR_LINEAR=$v: $(tail -1 $OUT/infer$v.log)"
done
AVR_LINEAR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 10 --warmup 3 > $OUT/prof1.log 2>&1 || { tail -20 $OUT/prof1.log; exit 1; }
python - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/linear/prof1/run_kernel_stats.csv')))[:6]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
