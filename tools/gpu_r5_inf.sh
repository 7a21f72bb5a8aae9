#!/bin/bash
# Round 5: inference small-kernel changes (bias kernel, unit map on load): tests, A/B, end to end.
set -u
OUT=gpurun_out/${1:-r5inf}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep "^{" $OUT/$name.log | tail -6 || true
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -25 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_hashgrid.py tests/test_gpu_sigma.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -2 $OUT/tests.log
L=tools/_lib
step xbias 300 python tools/xbench_bias.py "base=$L/libvar_hbase.so,v1=$L/libvar_hv1.so"
step infer 600 python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 30
echo all-ok
