#!/bin/bash
# Round 4 exact head / linear iteration: correctness of the pipelined exact
# head (variant 10) and the linear kernel, kernel stats, phase probes.
set -u
OUT=gpurun_out/hs3
mkdir -p $OUT
export TMPDIR=/tmp
AVR_EXACT_WAVES_PROBE=10 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $OUT/lin_tests.log 2>&1 || { tail -30 $OUT/lin_tests.log; exit 1; }
tail -1 $OUT/lin_tests.log
AVR_LINEAR_CT_PROBE=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $OUT/lin_tests32.log 2>&1 || { tail -30 $OUT/lin_tests32.log; exit 1; }
tail -1 $OUT/lin_tests32.log
timeout -k 10 200 python tools/probe_linear.py --dtype fp16 --reps 2 > $OUT/probe_lin.log 2>&1 || { tail -20 $OUT/probe_lin.log; exit 1; }
grep '^{' $OUT/probe_lin.log
for v in 8 10; do
  AVR_EXACT_WAVES_PROBE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$v -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof$v.log 2>&1 || { tail $OUT/prof$v.log; exit 1; }
  python - $v <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/hs3/prof{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:1]:
    print(sys.argv[1], r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
done
AVR_EXACT_WAVES_PROBE=10 timeout -k 10 200 python tools/probe_phases.py exact > $OUT/phases_exact.log 2>&1 || { tail -20 $OUT/phases_exact.log; exit 1; }
grep '^{' $OUT/phases_exact.log
timeout -k 10 200 python tools/probe_phases.py linear > $OUT/phases_linear.log 2>&1 || { tail -20 $OUT/phases_linear.log; exit 1; }
grep '^{' $OUT/phases_linear.log
timeout -k 10 400 python tools/ddp_buckets.py --steps 3 > $OUT/ddp_buckets.log 2>&1 || { tail -20 $OUT/ddp_buckets.log; exit 1; }
tail -2 $OUT/ddp_buckets.log
