#!/bin/bash
# h-stationary exact head (round 4): head tests, then kernel stats of the
# config-2 fp16 render through the exact head, per variant.
set -u
OUT=gpurun_out/hs
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for v in ${HS_VARIANTS:-8 4}; do
  AVR_EXACT_WAVES_PROBE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$v -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof$v.log 2>&1 || { tail $OUT/prof$v.log; exit 1; }
  python - $v <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/hs/prof{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:3]:
    print(sys.argv[1], r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
done
