#!/bin/bash
# Hash-grid backward with the reduce changes: parity tests, the whole
# partitioned backward against the previous build (configs 3 and 4), and
# the config-3 training step with kernel stats.
set -u
OUT=gpurun_out/${1:-hgred}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 600 python -u -m pytest tests/test_gpu_hashgrid.py tests/test_gpu_training.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
for w in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
  step xb_$w 300 python tools/xbench_hgbwd.py old=tools/_lib/libab_hg_old.so,cur=avr_amd/libavr_hip.so --workload $w --rounds 6 --iters 10
  grep "^{" $OUT/xb_$w.log
done
step train3 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
grep "^{" $OUT/train3.log | tail -1
step stats 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
echo all-ok
