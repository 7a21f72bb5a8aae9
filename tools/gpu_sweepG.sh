# Forward-reduction sweeps at G = 1: rows in flight (u4nt/u8nt) x ray splits.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export AVR_REDUCE_G=1
timeout -k 10 300 python tools/tune.py --variants u4nt,u8nt --nsplit 2,4 --ksplit 8 --rounds 5 --poses 16 > gpurun_out/sweepV_c2.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/tune.py --dtype float16 --variants u4nt,u8nt --nsplit 4,8,16 --ksplit 8 --rounds 3 --poses 16 > gpurun_out/sweepV_c2h.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/tune.py --workload c3_raf_furnished_b4 --variants u4nt,u8nt --nsplit 2,4 --ksplit 8 --rounds 3 > gpurun_out/sweepV_c3.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/tune.py --workload c5_simu_4096x512x2048 --variants u4nt,u8nt --nsplit 1,2,4 --ksplit 8 --rounds 2 --steps 5 --poses 4 > gpurun_out/sweepV_c5.jsonl 2>&1 || exit 1
