#!/bin/bash
set -u
OUT=gpurun_out/${1:-r5lin}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep "^{" $OUT/$name.log | tail -6 || true
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -25 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step lintest 300 python -u -m pytest tests/test_gpu_linear512.py -x -q --timeout 120 --timeout-method thread -W ignore
tail -2 $OUT/lintest.log
step linbench 300 python tools/bench_linear512.py --rows 262144,2097152 --dtype fp16 ${LIBS:+--libs $LIBS}
step linbench_bf 300 python tools/bench_linear512.py --rows 262144 --dtype bf16
echo all-ok
