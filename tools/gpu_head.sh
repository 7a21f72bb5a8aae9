# Fused-head tests and the head kernels' timings (one GPU session).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/h_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/h_tests.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hprof -o run --output-format csv -- python tools/bench_infer.py --steps 10 --warmup 3 > gpurun_out/h_prof.log 2>&1 || exit 1
tail -2 gpurun_out/h_prof.log
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/hprof/run_kernel_stats.csv')))
for r in rows[:14]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
