#!/bin/bash
# Band head phase timing under rocprofv3: AVR_HEAD_BAND_DBG 0 (full),
# 2 (no C terms), 8 (no band products), 10 (neither: the streaming skeleton);
# results of the switched-off runs are wrong by design.
set -u
OUT=gpurun_out/band
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/dbg -o run --output-format csv -- python tools/probe_band.py --dtype fp16 --forms 1 --dbgs ${DBGS:-0,2,8,10} > $OUT/dbg.log 2>&1 || { tail -20 $OUT/dbg.log; exit 1; }
python tools/trace_band.py $OUT/dbg/run_kernel_trace.csv ${DBGS:-0,2,8,10}
