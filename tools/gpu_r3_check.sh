#!/bin/bash
# Round-3 check: the tests touched this round, then the driver's bench command.
set -u
OUT=gpurun_out/r3check
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -W ignore \
  tests/test_gpu_head.py::test_fused_head_one_ray_shard tests/test_gpu_head.py::test_fused_head_propagate_nonfinite \
  tests/test_gpu_graph.py tests/test_gpu_render.py tests/test_gpu_training.py tests/test_gpu_bench_ranks.py \
  > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/drv$i.log; exit 1; }
  tail -1 $OUT/drv$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('drv', d['value'], d['ms_per_step'], d['ms_per_step_eager'], d['ir_render_ms_per_pose'], d['host_issue_ms_per_step'], d['roofline']['avg_launch_ms'], d['network_inference']['ms_per_pose'])"
done
