#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.
# Stops at the first crash/timeout (exit >= 124 or signal); test assertion
# failures (pytest exit 1) do not stop the later steps.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    modes) step bench_rayshard 300 python bench.py --mode ray-shard --steps 20 --warmup 3 --poses 4 \
           && step bench_ddp 300 python bench.py --mode ddp-train --steps 10 --warmup 3 \
           && step bench_gpus2 120 python bench.py --gpus 2 --steps 5 ;;
    newtests) step pytest_new 600 python -u -m pytest tests/test_gpu_dist2.py tests/test_gpu_reentrancy.py tests/test_gpu_graph.py "tests/test_gpu_render.py::test_nonfinite_semantics" -q -rf --timeout 120 --timeout-method thread ;;
    benchq) step bench_q 300 python bench.py --no-cpu-baseline --steps 100 ;;
    streams) step bench_s1 200 python bench.py --no-cpu-baseline --steps 200 --streams 1 && step bench_s2 200 python bench.py --no-cpu-baseline --steps 200 --streams 2 && step bench_s3 200 python bench.py --no-cpu-baseline --steps 200 --streams 3 ;;
    tune) step tune 600 python tools/tune.py ;;
    tune5) step tune5 600 python tools/tune.py --workload c5_simu_4096x512x2048 --rounds 3 --steps 5 --nsplit 2,4,8 --ksplit 8 --variants u4nt,u8nt,u4 ;;
    sweep) step sw_c2 300 python tools/tune.py --variants u4nt,u8nt --nsplit 1,2,4 --ksplit 8 --rounds 3 \
            && step sw_c2h 300 python tools/tune.py --dtype float16 --variants u4nt,u8nt --nsplit 2,4,8 --ksplit 8 --rounds 3 \
            && step sw_c3 300 python tools/tune.py --workload c3_raf_furnished_b4 --variants u4nt,u8nt --nsplit 2,4,8 --ksplit 8 --rounds 3 \
            && step sw_c5 300 python tools/tune.py --workload c5_simu_4096x512x2048 --variants u4nt,u8nt --nsplit 1,2,4,8 --ksplit 8 --rounds 2 --steps 5 \
            && step sw_c1 300 python tools/tune.py --workload c1_meshrir_plumbing --variants u4nt --nsplit 1,2,4 --ksplit 4 --rounds 3 ;;
    exp5) step exp_c2h 300 python tools/tune.py --dtype float16 --variants u4nt,u4 --nsplit 2,4 --ksplit 8 --rounds 3 \
            && step exp_c5_4088 300 python tools/tune.py --workload c5_simu_4096x512x2048 --T 4088 --variants u4nt,u4 --nsplit 4,8 --ksplit 8 --rounds 2 --steps 5 \
            && step exp_c5_S128 300 python tools/tune.py --workload c5_simu_4096x512x2048 --S 128 --variants u4nt,u4 --nsplit 4,8 --ksplit 8 --rounds 2 --steps 5 \
            && step exp_c5_fp32 300 python tools/tune.py --workload c5_simu_4096x512x2048 --S 128 --dtype float32 --variants u4nt --nsplit 2,4,8 --ksplit 8 --rounds 2 --steps 5 ;;
    train) step train_c3 600 python tools/bench_train.py && step train_c4 600 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu ;;
    trainu) step trainu_c3 600 python tools/bench_train.py --no-fused && step trainu_c4 600 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu --no-fused ;;
    wgrad) for v in 1 262144 500000 819200 100000000; do AVR_WGRAD_MIN=$v step wgrad_$v 300 python tools/bench_train.py --steps 10 || exit 1; done ;;
    infer) step infer_bf16 600 python tools/bench_infer.py && step infer_fp32 600 python tools/bench_infer.py --mlp-dtype fp32 ;;
    profinfer) step profinfer 600 rocprofv3 --kernel-trace --stats -d $OUT/profinfer -o run --output-format csv -- python tools/bench_infer.py --steps 5 --warmup 2 ;;
    torchprof) step torchprof 600 python tools/bench_train.py --steps 5 --profile ;;
    proftrain) step proftrain 600 rocprofv3 --kernel-trace --stats -d $OUT/proftrain -o run --output-format csv -- python tools/bench_train.py --steps 5 --warmup 2 ;;
    gexp) step g1 200 python tools/tune.py --variants u4nt --nsplit 2,4 --ksplit 8 --rounds 3 \
          && AVR_REDUCE_G=2 step g2 200 python tools/tune.py --variants u4nt --nsplit 1,2,4 --ksplit 8 --rounds 3 \
          && AVR_REDUCE_G=4 step g4 200 python tools/tune.py --variants u4nt --nsplit 1,2 --ksplit 8 --rounds 3 ;;
    tunebwd) step tunebwd 600 python tools/tune_bwd.py $TUNE_ARGS && step tunebwd2 600 python tools/tune_bwd.py --workload c2_meshrir_1024x256x512 $TUNE_ARGS && step tunebwd5 600 python tools/tune_bwd.py --workload c5_simu_4096x512x2048 $TUNE_ARGS ;;
    profcore) step profcore 600 rocprofv3 --kernel-trace --stats -d $OUT/profcore -o run --output-format csv -- python tools/bench_train.py --core-only --steps 20 ;;
    prof5) step prof5 600 rocprofv3 --kernel-trace --stats -d $OUT/prof5 -o run --output-format csv -- python bench.py --workload c5_simu_4096x512x2048 --no-cpu-baseline --steps 10 --warmup 2 --streams 1 --poses 4 ;;
    benchall) for wl in c1_meshrir_plumbing c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu c5_simu_4096x512x2048; do step bench_$wl 300 python bench.py --workload $wl --no-cpu-baseline --steps 50 || exit 1; done ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --streams 1 ;;
    pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 3 --streams 1 && step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 3 --streams 1 ;;
  esac
done
