#!/bin/bash
# Exact head with two t-tiles per wave (AVR_HEAD_EXACT_WAVES 20): the head
# tests under it, then kernel times against the persistent default (19),
# alternating, rocprofv3 kernel stats.
set -u
OUT=gpurun_out/w2
mkdir -p $OUT
export TMPDIR=/tmp
AVR_HEAD_EXACT_WAVES=20 timeout -k 10 600 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 120 --timeout-method thread -k "exact or config2 or model" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for wv in 19 20 19 20; do
  AVR_HEAD_EXACT_WAVES=$wv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p$wv -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 40 > $OUT/p$wv.log 2>&1 || { tail -20 $OUT/p$wv.log; exit 1; }
  python - $OUT/p$wv/run_kernel_stats.csv $wv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "head_exact" in r["Name"]:
        print("waves", sys.argv[2], r["Name"][:50], round(float(r["AverageNs"]) / 1000, 1), "us", r["Calls"])
PY
done
