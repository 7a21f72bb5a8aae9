# Fused-head and training tests (one GPU session).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/h_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/h_tests.log | head -20; exit $rc; }
