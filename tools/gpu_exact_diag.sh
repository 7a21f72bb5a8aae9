#!/bin/bash
# Exact head diagnosis at config 2 fp16: kernel stats, phase clocks (probe
# build), SQ counters.
set -u
OUT=gpurun_out/exact_diag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/exact_diag/prof/run_kernel_stats.csv')))[:3]:
    print(r['Name'][:80], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
timeout -k 10 200 python tools/probe_phases.py exact > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
grep '^{' $OUT/phases.log | tail -2
bash tools/pmc_exact.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
cat $OUT/pmc.log | grep -v "^W2\|^E2" | tail -20
