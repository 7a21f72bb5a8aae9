#!/bin/bash
# Fused finalize + irfft: render / graph tests, the driver's bench command,
# and a kernel trace of it (launches per pose, serial timeline).
set -u
OUT=gpurun_out/specir
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_render.py tests/test_gpu_graph.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network > $OUT/drv$i.log 2>&1 || { tail -20 $OUT/drv$i.log; exit 1; }
  tail -1 $OUT/drv$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('drv', d['value'], d['ms_per_step'], d['ms_per_step_eager'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
echo traced
