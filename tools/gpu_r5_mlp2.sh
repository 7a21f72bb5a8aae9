#!/bin/bash
# Round 5: hazard probe (interleaved-chain cases), fused-MLP variant A/B.
set -u
OUT=gpurun_out/${1:-r5mlp2}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  grep "^{" $OUT/$name.log || true
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -25 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step hazard 120 tools/_hazard_probe
L=tools/_lib
step xmlp 300 python tools/xbench_mlp.py "base=$L/libvar_mbase.so,dma=$L/libvar_mdma.so,nostage=$L/libvar_mnostage.so,nobar=$L/libvar_mnobar.so,nostore=$L/libvar_mnostore.so,dmanobar=$L/libvar_mdmanobar.so,noall=$L/libvar_mnoall.so"
step mlptest 300 python -u -m pytest tests/test_gpu_mlp512.py -x -q --timeout 120 --timeout-method thread -W ignore
echo all-ok
