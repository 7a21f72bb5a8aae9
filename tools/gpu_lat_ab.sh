#!/bin/bash
# Serial IR-render kernel timeline (graph replay), round-3 library (_ab_r3/) vs the current one.
set -u
OUT=$PWD/gpurun_out/lat_ab
mkdir -p $OUT
export TMPDIR=/tmp
for t in r3 r4; do
  d=.; [ $t = r3 ] && d=_ab_r3
  for m in graph eager; do
    flag=""; [ $m = eager ] && flag="--eager"
    (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$t$m -o run --output-format csv -- python tools/lat_trace.py $flag) > $OUT/$t$m.log 2>&1 || { tail $OUT/$t$m.log; exit 1; }
    echo "== $t $m $(grep latency_ms $OUT/$t$m.log)"
    python tools/lat_trace.py --report $(ls $OUT/$t$m/*/run_kernel_trace.csv $OUT/$t$m/run_kernel_trace.csv 2>/dev/null | head -1) | tail -9
  done
done
