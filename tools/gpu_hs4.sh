#!/bin/bash
# Exact head variants: 128-ray items, two workgroups per CU (default);
# 256-ray items (AVR_EXACT_RAYS_PROBE=256); 256-ray items with 64-t tiles
# (+ AVR_EXACT_TT_PROBE=64): tests, kernel stats, phase probes.
set -u
OUT=gpurun_out/hs4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for v in "256 32" "256 64"; do
  set -- $v
  AVR_EXACT_RAYS_PROBE=$1 AVR_EXACT_TT_PROBE=$2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py -k "k512 or config2 or many_rays" > $OUT/tests_$1_$2.log 2>&1
  rc=$?; tail -1 $OUT/tests_$1_$2.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests_$1_$2.log | head -30; exit $rc; }
done
for v in "128 32" "256 32" "256 64"; do
  set -- $v
  AVR_EXACT_RAYS_PROBE=$1 AVR_EXACT_TT_PROBE=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$1_$2 -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof$1_$2.log 2>&1 || { tail $OUT/prof$1_$2.log; exit 1; }
  python - $1_$2 <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/hs4/prof{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:1]:
    print(sys.argv[1], r['Name'][:70], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
  AVR_EXACT_RAYS_PROBE=$1 AVR_EXACT_TT_PROBE=$2 timeout -k 10 200 python tools/probe_phases.py exact > $OUT/phases$1_$2.log 2>&1 || { tail -20 $OUT/phases$1_$2.log; exit 1; }
  grep '^{' $OUT/phases$1_$2.log | tail -1
done
for sh in 0 1 2; do
  AVR_LINEAR_SHAPE_PROBE=$sh timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $OUT/lin_tests$sh.log 2>&1 || { tail -30 $OUT/lin_tests$sh.log; exit 1; }
  tail -1 $OUT/lin_tests$sh.log
done
timeout -k 10 300 python tools/probe_linear.py --dtype fp16 --reps 2 > $OUT/probe_lin.log 2>&1 || { tail -20 $OUT/probe_lin.log; exit 1; }
grep '^{' $OUT/probe_lin.log
AVR_LINEAR_SHAPE_PROBE=0 timeout -k 10 200 python tools/probe_phases.py linear > $OUT/phases_lin0.log 2>&1 || { tail -20 $OUT/phases_lin0.log; exit 1; }
grep '^{' $OUT/phases_lin0.log | tail -1
timeout -k 10 400 python tools/ddp_buckets.py --steps 3 > $OUT/ddp_buckets.log 2>&1 || { tail -20 $OUT/ddp_buckets.log; exit 1; }
tail -2 $OUT/ddp_buckets.log
timeout -k 10 200 python tools/lat_probe.py > $OUT/lat_probe.log 2>&1 || { tail -20 $OUT/lat_probe.log; exit 1; }
tail -1 $OUT/lat_probe.log
