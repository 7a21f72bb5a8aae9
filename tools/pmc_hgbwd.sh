#!/bin/bash
# Counter passes over the partitioned hash-grid backward (tools/xbench_hgbwd.py,
# the product library, config 3), one rocprofv3 --pmc run per pass.
set -u
OUT=${1:-gpurun_out/pmc_hg}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT" \
            "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"; do
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python tools/xbench_hgbwd.py cur=avr_amd/libavr_hip.so --rounds 1 --iters 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python - $OUT <<'PY'
import csv, glob, sys, statistics, json
d = sys.argv[1]
agg = {}
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hg_" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[-50:]
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, c in agg.items():
    print(json.dumps({"kernel": k, **{n: statistics.median(v) for n, v in c.items()}}))
PY
