#!/bin/bash
# Counter passes over config-2 fp16 inference (tools/bench_infer.py, fused
# path): SQ occupancy / LDS / MFMA, TCC hit rates, FETCH_SIZE, WRITE_SIZE,
# one rocprofv3 --pmc run per pass; then python tools/pmc_kernels.py.
set -u
OUT=${1:-gpurun_out/pmc_infer}
mkdir -p $OUT
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 4 --warmup 2"}
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
            "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES" \
            "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum" \
            "FETCH_SIZE" \
            "WRITE_SIZE"; do
  timeout -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python tools/pmc_kernels.py $OUT
