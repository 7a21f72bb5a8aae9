#!/bin/bash
# SQ counter passes over the exact fused head (tools/probe_exact_head.py,
# exact form only), one rocprofv3 --pmc run per pass.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/pmc_ex$i -o run --output-format csv -- python tools/probe_exact_head.py --modes exact --iters 5 > gpurun_out/pmc_ex$i.log 2>&1 || exit 1
  i=$((i+1))
done
python - <<'PY'
import csv, glob, collections
for i in range(2):
    for f in glob.glob(f'gpurun_out/pmc_ex{i}/**/*counter_collection.csv', recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if 'head_exact' in r['Kernel_Name']:
                acc[r['Counter_Name']].append(float(r['Counter_Value']))
        for k, v in sorted(acc.items()):
            print(k, sum(v) / max(1, len(v) // max(1, len(set([len(v)])))), len(v))
PY
