#!/bin/bash
# Persistent exact head (AVR_HEAD_EXACT_WAVES=19) against the one-item DMA
# form (17): head tests under 19, then kernel stats of both forms.
set -u
OUT=gpurun_out/persist
mkdir -p $OUT
export TMPDIR=/tmp
AVR_HEAD_EXACT_WAVES=19 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for w in 17 19; do
  AVR_HEAD_EXACT_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$w -o run --output-format csv -- python tools/probe_exact_head.py --modes exact > $OUT/prof$w.log 2>&1 || { tail $OUT/prof$w.log; exit 1; }
  python - $w <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/persist/prof{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:3]:
    print(sys.argv[1], r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
done
