#!/bin/bash
# bf16x3 DFT repro (tools/bf3_repro.sh built the libraries) and the GPU tests.
set -u
OUT=gpurun_out/${1:-r5bf3}
mkdir -p $OUT
timeout -k 10 300 python tools/bf3_repro.py --repeat 20 > $OUT/bf3.log 2>&1; rc=$?
cat $OUT/bf3.log | grep "^{" ; [ $rc -ne 0 ] && { tail -20 $OUT/bf3.log; exit $rc; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; exit $rc
