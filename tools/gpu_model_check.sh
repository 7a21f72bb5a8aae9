#!/bin/bash
# Model-side GPU tests with hipBLASLt hidden layers (default) and with the
# HIP GEMM (AVR_LINEAR=1).
set -u
OUT=gpurun_out/modelcheck
mkdir -p $OUT
export TMPDIR=/tmp
for v in 0 1; do
  AVR_LINEAR=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_sigma.py tests/test_gpu_training.py tests/test_gpu_linear.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $OUT/t$v.log 2>&1 || { tail -30 $OUT/t$v.log; exit 1; }
  echo "AVR_LINEAR=$v: $(tail -1 $OUT/t$v.log)"
done
