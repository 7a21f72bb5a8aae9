#!/bin/bash
# SQ counters of the config-3 training step's kernels (tools/bench_train.py),
# one rocprofv3 --pmc run.  bash tools/pmc_train.sh <out dir>
set -u
OUT=${1:-gpurun_out/pmc_train}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $OUT/p0 -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 5 --warmup 2 > $OUT/p0.log 2>&1 || { echo failed; tail -5 $OUT/p0.log; exit 1; }
echo ok
