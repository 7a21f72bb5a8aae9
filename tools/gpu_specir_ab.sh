#!/bin/bash
# A/B of the render_ir tail on one box: finalize + irfft (two launches)
# against avr_spectrum_ir (one launch), the driver's bench command, interleaved.
set -u
OUT=gpurun_out/specir_ab
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in 0 1; do
    AVR_SPECTRUM_IR=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline > $OUT/v$v.$i.log 2>&1 || { tail -20 $OUT/v$v.$i.log; exit 1; }
    tail -1 $OUT/v$v.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('v$v', d['value'], d['ms_per_step'], d['ms_per_step_eager'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'])"
  done
done
