#!/bin/bash
# Round 5: fused two-layer MLP (tests + A/B), bf16x3 DFT repro, all GPU tests.
set -u
OUT=gpurun_out/${1:-r5mlp}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep "^{" $OUT/$name.log || true
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -25 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step mlptest 300 python -u -m pytest tests/test_gpu_mlp512.py -x -q --timeout 120 --timeout-method thread -W ignore
tail -2 $OUT/mlptest.log
step mlpbench 300 python tools/bench_mlp512.py --rows 262144,2097152 --dtype fp16
step bf3 300 python tools/bf3_repro.py --repeat 20
if [ "${FULL:-1}" = 1 ]; then
  step tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
  tail -2 $OUT/tests.log
fi
echo all-ok
