#!/bin/bash
# PyTorch TunableOp tuning of the library GEMMs of config-2 inference (the
# width-512 hidden layers, hipBLASLt / rocBLAS candidates) for fp16 and bf16
# MLPs; the results file is what avr_amd/tunableop_gfx950.csv ships
# (avr_amd/model.py: _enable_tuned_gemms).
set -u
OUT=gpurun_out/tune
mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/tunableop_gfx950*.csv
# TRAIN=1: only the training shapes, added to the shipped inference results;
# C5=1: only config 5's (2,097,152-row width-512 layers, fp16), likewise
if [ "${C5:-0}" = 1 ]; then
  cp avr_amd/tunableop_gfx950.csv $OUT/tunableop_gfx950.csv
  (export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv; timeout -k 10 900 python bench.py --mode ray-shard --network --mlp-dtype ${C5_DTYPE:-fp16} --steps 1 --warmup 1 --no-cpu-baseline) > $OUT/tune_c5.log 2>&1 || { tail -20 $OUT/tune_c5.log; exit 1; }
  cat $OUT/tunableop_gfx950*.csv
  exit 0
fi
[ "${TRAIN:-0}" = 1 ] && cp avr_amd/tunableop_gfx950.csv $OUT/tunableop_gfx950.csv
for dt in fp16 bf16; do
  [ "${TRAIN:-0}" = 1 ] && break
  (export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv; timeout -k 10 500 python tools/bench_infer.py --mlp-dtype $dt --variants fused --steps 2 --warmup 1) > $OUT/tune_$dt.log 2>&1 || { tail -20 $OUT/tune_$dt.log; exit 1; }
done
[ "${TRAIN:-0}" = 1 ] || { ls $OUT; cat $OUT/tunableop_gfx950*.csv; }
# the training steps of configs 3 and 4 (bf16 MLPs: forward, data and weight gradients)
if [ "${TRAIN:-0}" = 1 ]; then
  for wl in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
    (export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv; timeout -k 10 500 python tools/bench_train.py --workload $wl --steps 2 --warmup 1) > $OUT/tune_$wl.log 2>&1 || { tail -20 $OUT/tune_$wl.log; exit 1; }
  done
  # TunableOp inserts the device ordinal into the name (tunableop_gfx9500.csv)
  cat $OUT/tunableop_gfx950*.csv
fi
