#!/bin/bash
# The width-512 hidden-layer GEMM: tests, then timing against hipBLASLt
# (both kernel variants interleaved), then kernel stats.
set -u
OUT=gpurun_out/linear
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AVR_LINEAR_WAVES_PROBE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $OUT/tests4.log 2>&1 || { tail -30 $OUT/tests4.log; exit 1; }
tail -1 $OUT/tests4.log
for d in fp16 bf16; do
  timeout -k 10 200 python tools/probe_linear.py --dtype $d --reps 3 > $OUT/probe_$d.log 2>&1 || { tail -20 $OUT/probe_$d.log; exit 1; }
  grep '^{' $OUT/probe_$d.log
done
