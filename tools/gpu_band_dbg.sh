#!/bin/bash
# Band head: partial check per ring shape, then phase timing
# (AVR_HEAD_BAND_DBG 0 / 10: no C term, no chunk compute) under rocprofv3.
set -u
OUT=gpurun_out/band
mkdir -p $OUT
export TMPDIR=/tmp
for rg in ${RINGS:-4 5}; do
  AVR_HEAD_BAND_RING=$rg timeout -k 10 200 python tools/probe_band_z.py --case raf --dtype bf16 --cols 4 --forms 1 > $OUT/z$rg.log 2>&1 || { tail -20 $OUT/z$rg.log; exit 1; }
  echo "ring $rg: $(grep -c '"n_bad": 0' $OUT/z$rg.log) of 4 columns exact"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/dbgr -o run --output-format csv -- python tools/probe_band.py --dtype fp16 --forms 1 --rings 0,4,5,6 --dbgs 0,10 > $OUT/dbgr.log 2>&1 || { tail -20 $OUT/dbgr.log; exit 1; }
python tools/trace_band.py $OUT/dbgr/run_kernel_trace.csv r0d0,r0d10,r4d0,r4d10,r5d0,r5d10,r6d0,r6d10
