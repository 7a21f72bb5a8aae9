#!/bin/bash
# Round 5: fused MLP check + exact-head v2 A/B (c2, c5), then the GPU suite.
set -u
FULL=0 bash tools/gpu_r5_mlp.sh ${1:-r5v2} || exit $?
LIBS="base=tools/_lib/libvar_base.so,v2=tools/_lib/libvar_v2.so" WORKLOADS="c2_meshrir_1024x256x512 c5_simu_4096x512x2048" \
  bash tools/gpu_xab.sh ${1:-r5v2}_xab || exit $?
if [ "${FULL:-1}" = 1 ]; then
  OUT=gpurun_out/${1:-r5v2}
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
echo all-ok
