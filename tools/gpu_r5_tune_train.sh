#!/bin/bash
# Tune the training GEMMs of configs 3 and 4 (TunableOp, TRAIN=1 of
# tune_gemms.sh), then time each MLP-backward shape's data gradient with and
# without the tuned solutions (tools/bench_wgrad.py --tuned).
set -u
OUT=gpurun_out/tunetrain
mkdir -p $OUT
TRAIN=1 timeout -k 10 900 bash tools/tune_gemms.sh > $OUT/tune.log 2>&1 || { tail -30 $OUT/tune.log; exit 1; }
cp gpurun_out/tune/tunableop_gfx950*.csv $OUT/ 2>/dev/null
F=$(ls gpurun_out/tune/tunableop_gfx950*.csv | head -1)
timeout -k 10 200 python tools/bench_wgrad.py --tuned $F > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 1; }
timeout -k 10 200 python tools/bench_wgrad.py --workload c4_raf_empty_b4_per_gpu --tuned $F > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 1; }
echo done
