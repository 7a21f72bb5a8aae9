#!/bin/bash
set -u
OUT=gpurun_out/r5stage
mkdir -p $OUT
L=tools/_lib
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep "^{" $OUT/$name.log | tail -4 || true
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -25 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 600 python -u -m pytest tests/test_gpu_sigma.py tests/test_gpu_linear512.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
step xsig 300 python tools/xbench_sigma.py "old=$L/libvar_sold.so,new=$L/libvar_sbase2.so" --rounds 8
step xsigbf 300 python tools/xbench_sigma.py "old=$L/libvar_sold.so,new=$L/libvar_sbase2.so" --rounds 8 --dtype bf16
step xlin 300 python tools/bench_linear512.py --rows 262144 --libs old=$L/libvar_lold.so --rounds 8
echo all-ok
