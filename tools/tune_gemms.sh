#!/bin/bash
# PyTorch TunableOp tuning of the library GEMMs of config-2 inference (the
# width-512 hidden layers, hipBLASLt / rocBLAS candidates) for fp16 and bf16
# MLPs; the results file is what avr_amd/tunableop_gfx950.csv ships
# (avr_amd/model.py: _enable_tuned_gemms).
set -u
OUT=gpurun_out/tune
mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/tunableop_gfx950.csv
for dt in fp16 bf16; do
  (export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_gfx950.csv AVR_TUNABLEOP=0; timeout -k 10 500 python tools/bench_infer.py --mlp-dtype $dt --variants fused --steps 2 --warmup 1) > $OUT/tune_$dt.log 2>&1 || { tail -20 $OUT/tune_$dt.log; exit 1; }
done
ls $OUT; cat $OUT/tunableop_gfx950*.csv
