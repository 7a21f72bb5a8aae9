#!/bin/bash
# Exact-head A/B of variant libraries (tools/xbench_exact.py) and phase probes
# of probe-build variants (tools/probe_phases.py), one GPU call.
#   LIBS="base=tools/_lib/libvar_base.so,x=..." PROBES="pbase pstag" bash tools/gpu_xab.sh OUT
set -u
OUT=gpurun_out/${1:-xab}
mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"; cat $OUT/$name.log | grep "^{" || true
}
for wl in ${WORKLOADS:-c2_meshrir_1024x256x512}; do
  step xab_$wl 400 python tools/xbench_exact.py "$LIBS" --workload $wl --rounds ${ROUNDS:-5} --iters ${ITERS:-10}
  # LIBS2: a second set (new, riskier variants), run only after the first passed
  if [ -n "${LIBS2:-}" ]; then
    step xab2_$wl 400 python tools/xbench_exact.py "$LIBS2" --workload $wl --rounds ${ROUNDS:-5} --iters ${ITERS:-10}
  fi
done
for p in ${PROBES:-}; do
  AVR_PROBE_LIB=tools/_lib/libvar_$p.so step probe_$p 300 python tools/probe_phases.py exact ${SKIPS:-0}
done
echo all-ok
