#!/bin/bash
# Default bench line (with the network-inference leg) + kernel stats of the
# fp16 reference-network inference.  Stops at the first failing step.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_net.log 2>&1 || { echo "bench rc=$?"; tail -20 $OUT/bench_net.log; exit 1; }
tail -1 $OUT/bench_net.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/profinfer16 -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 10 --warmup 3 > $OUT/profinfer16.log 2>&1 || { echo "prof rc=$?"; tail -20 $OUT/profinfer16.log; exit 1; }
tail -1 $OUT/profinfer16.log
