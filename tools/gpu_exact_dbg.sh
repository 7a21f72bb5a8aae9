#!/bin/bash
# Exact head, the one-item LDS-DMA form with 64-ray tiles (AVR_HEAD_EXACT_WAVES
# 17) under phase switches (AVR_HEAD_EXACT_DBG: 0 full, 5 the row stream
# alone: no MFMA, no epilogue; 12 MFMA chains alone: no epilogue, no DMA),
# and the persistent default (19), rocprofv3 kernel trace.
set -u
OUT=gpurun_out/exactdbg
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "19 0" "17 0" "17 5" "17 12"; do
  set -- $cfg
  AVR_HEAD_EXACT_WAVES=$1 AVR_HEAD_EXACT_DBG=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/w$1d$2 -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 20 > $OUT/w$1d$2.log 2>&1 || { tail -20 $OUT/w$1d$2.log; exit 1; }
  python - $OUT/w$1d$2/run_kernel_stats.csv "$1 $2" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "head_exact" in r["Name"]:
        print("waves/dbg", sys.argv[2], r["Name"][:60], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
done
