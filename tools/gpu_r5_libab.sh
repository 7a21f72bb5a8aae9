#!/bin/bash
# Training-step A/B across whole-library builds (tools/_lib/libvar_<name>.so,
# every source): each is copied over the box's snapshot of the product
# library in turn, interleaved twice.  Usage: tools/gpu_r5_libab.sh name ...
set -u
OUT=gpurun_out/${TAG:-libab}
mkdir -p $OUT
cp avr_amd/libavr_hip.so $OUT/product.so
for rep in 1 2; do
  for v in "$@"; do
    cp tools/_lib/libvar_$v.so avr_amd/libavr_hip.so
    for wl in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
      timeout -k 10 200 python tools/bench_train.py --workload $wl --steps ${STEPS:-40} > $OUT/${wl}_${v}_$rep.log 2>&1 || { tail -20 $OUT/${wl}_${v}_$rep.log; cp $OUT/product.so avr_amd/libavr_hip.so; exit 1; }
      tail -1 $OUT/${wl}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $v $rep', round(d['train_step_ms'],3))"
    done
  done
done
cp $OUT/product.so avr_amd/libavr_hip.so
