set -u
mkdir -p gpurun_out/r5sync
timeout -k 10 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 3 --warmup 2 --sync-debug > gpurun_out/r5sync/c3.log 2>&1; rc=$?
grep -c "SYNC:" gpurun_out/r5sync/c3.log; grep -A16 "SYNC:" gpurun_out/r5sync/c3.log | head -120; exit $rc
