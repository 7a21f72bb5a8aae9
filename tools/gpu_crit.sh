#!/bin/bash
# Criterion loss total in the reduce kernel: criterion / training / DAS tests and the
# config-3 and config-4 training steps with kernel stats.
set -u
OUT=gpurun_out/${1:-crit}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 900 python -u -m pytest tests/test_gpu_criterion.py tests/test_gpu_training.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
step train3 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
grep "^{" $OUT/train3.log | tail -1
step train4 300 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu --steps 30
grep "^{" $OUT/train4.log | tail -1
step stats 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
echo all-ok
