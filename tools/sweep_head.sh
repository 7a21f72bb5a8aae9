#!/bin/bash
# Head-forward variants at config 2 (and 3): AVR_HEAD_RING x AVR_HEAD_SB, kernel
# times from rocprofv3 kernel traces (gpurun_out/sh_*/).
set -u
export TMPDIR=/tmp
for wl in ${WLS:-c2_meshrir_1024x256x512}; do
for ring in ${RINGS:-0 1}; do for sb in ${SBS:-2 4}; do
  d=gpurun_out/sh_${wl}_r${ring}_s${sb}
  AVR_HEAD_RING=$ring AVR_HEAD_SB=$sb timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python tools/probe_head.py --workload $wl --dbg ${DBGS:-0,5} --iters 5 > $d.log 2>&1 || exit 1
done; done; done
