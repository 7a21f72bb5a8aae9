#!/bin/bash
# Round 5: hash-grid backward written not added, sigma ReLU form; tests, A/B.
set -u
OUT=gpurun_out/${1:-r5train}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep "^{" $OUT/$name.log | tail -4 || true
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -25 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 900 python -u -m pytest tests/test_gpu_hashgrid.py tests/test_gpu_sigma.py tests/test_gpu_training.py tests/test_gpu_mlp512.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -2 $OUT/tests.log
L=tools/_lib
step xsig16 300 python tools/xbench_sigma.py "base=$L/libvar_sbase.so,relu0=$L/libvar_srelu0.so"
step xsig_bf 300 python tools/xbench_sigma.py "base=$L/libvar_sbase.so,relu0=$L/libvar_srelu0.so" --dtype bf16
for w in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
  step tr_${w}_set 400 python tools/bench_train.py --workload $w --steps 20
  AVR_HASHGRID_BWD=partitioned_add step tr_${w}_add 400 python tools/bench_train.py --workload $w --steps 20
  step tr_${w}_set2 400 python tools/bench_train.py --workload $w --steps 20
done
echo all-ok
