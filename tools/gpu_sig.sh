#!/bin/bash
# Sigma h1 kernel A/B: parity tests, isolated timing against the previous
# build (tools/_lib/libab_sig_old.so) per tile config, SQ counters,
# config-2 inference.
set -u
OUT=gpurun_out/${1:-sig}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 600 python -u -m pytest tests/test_gpu_sigma.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
step xb 300 python tools/xbench_sigma.py old=tools/_lib/libab_sig_old.so:identity:0 cur=avr_amd/libavr_hip.so:stream:0,11,12,14 --rounds 6
cat $OUT/xb.log | grep "^{"
step pmc 400 bash tools/pmc_sigma.sh 2 0,11,12 $OUT/pmc
grep "^{" $OUT/pmc.log
echo all-ok
