#!/bin/bash
# h-stationary exact head: kernel stats of the 8-wave form with plain (8) and
# non-temporal (9) h loads, then PMC passes (HBM bytes, L2 hit rate, SQ) on
# both; then the x-stationary linear kernel's tests and A/B timing.
set -u
OUT=gpurun_out/hs2
mkdir -p $OUT
export TMPDIR=/tmp
for v in 8 9; do
  AVR_EXACT_WAVES_PROBE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$v -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 30 > $OUT/prof$v.log 2>&1 || { tail $OUT/prof$v.log; exit 1; }
  python - $v <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/hs2/prof{sys.argv[1]}/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:2]:
    print(sys.argv[1], r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
done
i=0
for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"; do
  for v in 8 9; do
    AVR_EXACT_WAVES_PROBE=$v timeout -s KILL 90 rocprofv3 --pmc $pass -d $OUT/pmc${i}_$v -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 5 > $OUT/pmc${i}_$v.log 2>&1 || { tail $OUT/pmc${i}_$v.log; exit 1; }
    echo "== pass $i variant $v"; python tools/pmc_read.py $OUT/pmc${i}_$v --match head_exact
  done
  i=$((i+1))
done
bash tools/gpu_linear.sh
