#!/bin/bash
# Register bitonic sort in head_sort: head/model parity tests, then timing.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_head.py tests/test_gpu_model.py tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $OUT/sort_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/sort_tests.log; exit 1; }
tail -1 $OUT/sort_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/profsort -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 10 --warmup 3 > $OUT/profsort.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/profsort.log; exit 1; }
tail -1 $OUT/profsort.log
timeout -k 10 120 python tools/gemm_layout_probe.py > $OUT/gemm_layout.log 2>&1 || { echo "gemm rc=$?"; tail -20 $OUT/gemm_layout.log; exit 1; }
cat $OUT/gemm_layout.log
