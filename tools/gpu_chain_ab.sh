#!/bin/bash
# Chunked inference ReLU chain (MLP._relu_chain) A/B in the bench's
# network-inference leg, plus the model / sigma / head tests.
set -u
OUT=gpurun_out/chain
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_model.py tests/test_gpu_sigma.py tests/test_gpu_graph.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2; do
  for v in 0 1; do
    AVR_CHAIN_CHUNKS=$v timeout -k 10 300 python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 20 > $OUT/inf$v.$i.log 2>&1 || { tail -20 $OUT/inf$v.$i.log; exit 1; }
    echo "chunks=$v $(tail -1 $OUT/inf$v.$i.log | cut -c1-300)"
  done
done
