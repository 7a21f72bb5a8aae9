export TMPDIR=/tmp; mkdir -p gpurun_out/tt
for v in 1 0 1 0; do
  AVR_TUNABLEOP=$v timeout -k 10 300 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu > gpurun_out/tt/c4_$v.log 2>&1 || { tail gpurun_out/tt/c4_$v.log; exit 1; }
  echo "tuned=$v $(tail -1 gpurun_out/tt/c4_$v.log | cut -c1-200)"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore -k "train or model or grad or ddp or dist" > gpurun_out/tt/tests.log 2>&1; rc=$?; tail -1 gpurun_out/tt/tests.log; exit $rc
