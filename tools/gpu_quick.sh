#!/bin/bash
# All GPU tests, then the default-config bench (1 and 2 streams).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -W ignore > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench2.log 2>&1 || exit 1
tail -1 gpurun_out/bench2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('2s', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['host_issue_ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --streams 1 > gpurun_out/bench1.log 2>&1 || exit 1
tail -1 gpurun_out/bench1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1s', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['host_issue_ms_per_step'], d['roofline']['avg_launch_ms'])"
