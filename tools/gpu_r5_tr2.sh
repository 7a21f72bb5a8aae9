set -u
mkdir -p gpurun_out/r5tr2
for w in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
timeout -k 10 400 python tools/bench_train.py --workload $w --steps 20 > gpurun_out/r5tr2/$w.log 2>&1 || { tail -20 gpurun_out/r5tr2/$w.log; exit 1; }
tail -1 gpurun_out/r5tr2/$w.log
done
