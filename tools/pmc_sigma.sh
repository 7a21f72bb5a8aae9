#!/bin/bash
# SQ counter passes over the fused sigma kernel (tools/probe_sigma.py on the
# product library), one rocprofv3 --pmc run per pass.
#   bash tools/pmc_sigma.sh <variant> <cfgs> <out dir>
set -u
V=${1:-2}; CFGS=${2:-0}; OUT=${3:-gpurun_out/pmc_sig}
export TMPDIR=/tmp AVR_AB_LIB=$PWD/avr_amd/libavr_hip.so
mkdir -p $OUT
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python tools/probe_sigma.py --variant $V --dtype fp16 --cfgs $CFGS --iters 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python - $OUT <<'PY'
import csv, glob, sys, statistics, json
d = sys.argv[1]
agg = {}
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "sigma" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[-60:]
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: statistics.median(v) for n, v in c.items()}
    print(json.dumps({"kernel": k, **m}))
PY
