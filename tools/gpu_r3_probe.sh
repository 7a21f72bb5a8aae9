#!/bin/bash
# Round-3 first probe: the driver's exact bench command twice, then a kernel
# trace of the same command (timestamps, to find the per-step gaps).
set -u
OUT=gpurun_out/r3probe
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network > $OUT/drv$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/drv$i.log; exit 1; }
  tail -1 $OUT/drv$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('drv', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['host_issue_ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
