#!/bin/bash
set -u
OUT=gpurun_out/${1:-r5mlp3}
mkdir -p $OUT
L=tools/_lib
timeout -k 10 300 python tools/xbench_mlp.py "base=$L/libvar_mbase.so,${LIBS}" > $OUT/xmlp.log 2>&1
rc=$?; cat $OUT/xmlp.log | grep "^{"; exit $rc
