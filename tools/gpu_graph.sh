# Graph tests, the latency probe and the default bench (one GPU session).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_render.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/g_tests.log | head -20; exit $rc; }
timeout -k 10 200 python tools/graph_probe.py > gpurun_out/g_probe.log 2>&1 || exit 1
tail -1 gpurun_out/g_probe.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/g_bench.log 2>&1 || exit 1
tail -1 gpurun_out/g_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], 'lat', d['ir_render_ms_per_pose'], 'eager', d['ir_render_ms_per_pose_eager'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
