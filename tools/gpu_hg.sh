#!/bin/bash
# Hash-grid grouped corner loads: parity tests, then A/B timing.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hashgrid.py -x -q --timeout 120 --timeout-method thread > $OUT/hg_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/hg_tests.log; exit 1; }
tail -1 $OUT/hg_tests.log
for g in 0 1 0 1; do
  AVR_HASHGRID_GROUP=$g timeout -k 10 120 python tools/probe_hashgrid.py > $OUT/hg_probe_$g.log 2>&1 || { echo "probe rc=$?"; tail -20 $OUT/hg_probe_$g.log; exit 1; }
  echo "group=$g"; cat $OUT/hg_probe_$g.log | grep dtype
done
for g in 0 1; do
  AVR_HASHGRID_GROUP=$g timeout -k 10 200 python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 30 > $OUT/hg_infer_$g.log 2>&1 || { echo "infer rc=$?"; tail -20 $OUT/hg_infer_$g.log; exit 1; }
  echo "group=$g"; tail -1 $OUT/hg_infer_$g.log
done
