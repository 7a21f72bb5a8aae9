set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --workload c5_simu_4096x512x2048 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_c5.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c5.log
timeout -k 10 200 python tools/bench_infer.py --variants fused --steps 30 > gpurun_out/infer.log 2>&1 || exit 1
tail -3 gpurun_out/infer.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o prof -- python bench.py --workload c5_simu_4096x512x2048 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof_c5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inf -o prof -- python tools/bench_infer.py --variants fused --steps 10 > gpurun_out/prof_inf.log 2>&1 || exit 1
