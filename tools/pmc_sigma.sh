#!/bin/bash
# SQ counter passes over the fused sigma kernel (tools/probe_sigma.py), one
# rocprofv3 --pmc run per pass.  Usage: bash tools/pmc_sigma.sh <cfgs>
set -u
CFGS=${1:-0}
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_IFETCH SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"; do
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/pmc_sig$i -o run --output-format csv -- python tools/probe_sigma.py --cfgs $CFGS --iters 5 > gpurun_out/pmc_sig$i.log 2>&1 || exit 1
  i=$((i+1))
done
