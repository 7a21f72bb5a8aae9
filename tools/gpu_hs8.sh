#!/bin/bash
# A/B of the persistent exact head against the previous build; the DFT tail
# (render tests + the serial IR timeline).
set -u
OUT=gpurun_out/hs8
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore -m gpu tests/test_gpu_render.py tests/test_gpu_graph.py tests/test_gpu_reentrancy.py tests/test_gpu_knobs.py tests/test_gpu_properties.py > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
timeout -k 10 300 python tools/ab_exact.py --rounds 6 --iters 20 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -1 $OUT/ab.log
AVR_EXACT_RAYS_PROBE=256 AVR_EXACT_TT_PROBE=64 timeout -k 10 300 python tools/ab_exact.py --rounds 6 --iters 20 > $OUT/ab256.log 2>&1 || { tail -20 $OUT/ab256.log; exit 1; }
tail -1 $OUT/ab256.log
bash tools/gpu_lat.sh
bash tools/pmc_infer.sh gpurun_out/pmc_infer > gpurun_out/hs8/pmc.log 2>&1 || { tail -20 gpurun_out/hs8/pmc.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hs8/infer_stats -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 20 > gpurun_out/hs8/infer.log 2>&1 || { tail gpurun_out/hs8/infer.log; exit 1; }
grep -i "ms" gpurun_out/hs8/infer.log | tail -3
timeout -k 10 400 python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/hs8/rayshard_net.log 2>&1 || { tail -20 gpurun_out/hs8/rayshard_net.log; exit 1; }
tail -1 gpurun_out/hs8/rayshard_net.log
