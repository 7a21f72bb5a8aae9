#!/bin/bash
# Exact-head iteration: its parity tests, kernel stats at config 2 fp16 and
# the probe build's phase clocks (skip masks $1, default "0,7").
set -u
OUT=gpurun_out/exact_iter
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore -m gpu tests/test_gpu_head.py -k "exact or config2 or many_rays" > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/exact_iter/prof/run_kernel_stats.csv')))[:2]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
mkdir -p $OUT/dump
AVR_PROBE_DUMP=$OUT/dump timeout -k 10 200 python tools/probe_phases.py exact ${1:-0,7} > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
python tools/exact_items.py $OUT/dump
