#!/bin/bash
# Serial IR-render kernel timeline (graph replay) under the validated tuning
# knobs: DFT k-slices (AVR_KSPLIT) and reduction ray splits (AVR_NSPLIT).
set -u
OUT=$PWD/gpurun_out/lat_knobs
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "AVR_KSPLIT=8" "AVR_KSPLIT=16" "AVR_KSPLIT=4" "AVR_NSPLIT=1" "AVR_NSPLIT=4"; do
  n=${kv//=/_}
  (export $kv; timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$n -o run --output-format csv -- python tools/lat_trace.py) > $OUT/$n.log 2>&1 || { tail $OUT/$n.log; exit 1; }
  echo "== $kv $(grep latency_ms $OUT/$n.log)"
  python tools/lat_trace.py --report $(ls $OUT/$n/*/run_kernel_trace.csv $OUT/$n/run_kernel_trace.csv 2>/dev/null | head -1) | tail -8
done
