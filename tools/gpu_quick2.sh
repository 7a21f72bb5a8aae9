# Render tests + 1/2-stream bench + kernel stats (one GPU session).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_graph.py tests/test_gpu_properties.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/q2_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/q2_tests.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/q2_bench2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --streams 1 > gpurun_out/q2_bench1.log 2>&1 || exit 1
for f in q2_bench2 q2_bench1; do tail -1 gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q2prof -o run --output-format csv -- python bench.py --no-cpu-baseline --streams 1 --steps 100 > gpurun_out/q2_prof.log 2>&1 || exit 1
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/q2prof/run_kernel_stats.csv')))
for r in rows[:9]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
