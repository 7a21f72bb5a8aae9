#!/bin/bash
# A/B of the render core against the round-3 library (_ab_r3/, built from
# 08a91af by hand, not committed): the driver's bench line without the
# network and CPU legs, interleaved.
set -u
OUT=gpurun_out/ab_r3
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  for t in r3 r4; do
    d=.; [ $t = r3 ] && d=_ab_r3
    (cd $d && timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-network --no-cpu-baseline) > $OUT/$t.$i.log 2>&1 || { tail -20 $OUT/$t.$i.log; exit 1; }
    tail -1 $OUT/$t.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', $i, round(d['ms_per_step'],4), round(d['ms_per_step_graph'],4), round(d['ir_render_ms_per_pose'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
