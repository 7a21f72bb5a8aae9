#!/bin/bash
# Exact head with the parallel prologue: tests, kernel stats and phases for
# the 128-ray and 256-ray/64-t variants; then the serial IR timeline.
set -u
OUT=gpurun_out/hs6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
AVR_EXACT_RAYS_PROBE=256 AVR_EXACT_TT_PROBE=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py -k "k512 or config2 or many_rays" > $OUT/tests_256_64.log 2>&1
rc=$?; tail -1 $OUT/tests_256_64.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests_256_64.log | head -30; exit $rc; }
for v in "128 32" "256 64"; do
  set -- $v
  AVR_EXACT_RAYS_PROBE=$1 AVR_EXACT_TT_PROBE=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$1_$2 -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof$1_$2.log 2>&1 || { tail $OUT/prof$1_$2.log; exit 1; }
  python - $1_$2 <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/hs6/prof{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:1]:
    print(sys.argv[1], r['Name'][:70], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
  AVR_EXACT_RAYS_PROBE=$1 AVR_EXACT_TT_PROBE=$2 timeout -k 10 200 python tools/probe_phases.py exact > $OUT/phases$1_$2.log 2>&1 || { tail -20 $OUT/phases$1_$2.log; exit 1; }
  grep '^{' $OUT/phases$1_$2.log | tail -1
done
