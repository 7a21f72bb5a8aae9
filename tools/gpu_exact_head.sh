#!/bin/bash
# Exact (MFMA) fused head: tests, then timing + kernel stats at config 2.
set -u
OUT=gpurun_out/exact
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python tools/probe_exact_head.py > $OUT/probe.log 2>&1 || { tail $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/probe_exact_head.py > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/exact/prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
