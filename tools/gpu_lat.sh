#!/bin/bash
# Kernel timeline of the serial IR render, graph replay and eager issue.
set -u
OUT=gpurun_out/lat
mkdir -p $OUT
export TMPDIR=/tmp
for m in graph eager; do
  flag=""; [ $m = eager ] && flag="--eager"
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$m -o run --output-format csv -- python tools/lat_trace.py $flag > $OUT/$m.log 2>&1 || { tail $OUT/$m.log; exit 1; }
  grep latency_ms $OUT/$m.log
  python tools/lat_trace.py --report $(ls $OUT/$m/*/run_kernel_trace.csv $OUT/$m/run_kernel_trace.csv 2>/dev/null | head -1) | tail -14
done
