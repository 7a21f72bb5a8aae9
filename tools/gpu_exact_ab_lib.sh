#!/bin/bash
# Exact head, current source against the previous build (libavr_shapes_old.so,
# built from the stashed tree by hand): head tests, then the config-2 fp16
# fused render timed in alternating processes.
set -u
OUT=gpurun_out/exact_ab_lib
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore -m gpu tests/test_gpu_head.py tests/test_gpu_model.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2 3; do
  for v in new old; do
    lib=tools/_lib/libavr_shapes.so; [ $v = old ] && lib=tools/_lib/libavr_shapes_old.so
    AVR_AB_LIB=$PWD/$lib timeout -k 10 200 python tools/ab_shapes.py --shapes 256/64 --rounds 3 > $OUT/$v.$i.log 2>&1 || { tail $OUT/$v.$i.log; exit 1; }
    echo "$v $i $(grep 'shape 256/64:' $OUT/$v.$i.log)"
  done
done
