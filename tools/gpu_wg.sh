#!/bin/bash
# Weight-gradient tile A/B: wgrad tests, the kernel against the previous
# build at the training shapes, the config-3 step with kernel stats.
set -u
OUT=gpurun_out/${1:-wg}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_training.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
step xb 300 python tools/xbench_wgrad.py old=tools/_lib/libab_wg_old.so,cur=avr_amd/libavr_hip.so
grep "^{" $OUT/xb.log
step train3 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
grep "^{" $OUT/train3.log | tail -1
echo all-ok
