#!/bin/bash
# Hash-grid backward A/B inside the config-3/4 training step: tests, then
# bench_train with the partitioned and the atomic backward, then a kernel
# profile of the default step.
set -o pipefail
OUT=gpurun_out/hgtrain
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hashgrid.py tests/test_gpu_training.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -W ignore > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for impl in partitioned atomic partitioned atomic; do
  AVR_HASHGRID_BWD=$impl timeout -k 10 300 python tools/bench_train.py --steps 30 > $OUT/bt_$impl.log 2>&1 || { tail -20 $OUT/bt_$impl.log; exit 1; }
  echo "$impl $(tail -1 $OUT/bt_$impl.log)"
done
timeout -k 10 300 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu > $OUT/bt_c4.log 2>&1 && tail -1 $OUT/bt_c4.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/bench_train.py --steps 5 --warmup 2 > $OUT/prof.log 2>&1 && echo profok
