#!/bin/bash
# Round 6: sigma h1 layer order + native clip coefficient: parity tests,
# config-2 inference with kernel stats, config-3 training with kernel stats.
set -u
OUT=gpurun_out/${1:-r6c}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 600 python -u -m pytest tests/test_gpu_sigma.py tests/test_gpu_training.py tests/test_gpu_model.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
step infer 300 python tools/bench_infer.py --mlp-dtype fp16 --variants fused --repeat 3 --steps 30
grep "^{" $OUT/infer.log
step inferstats 400 rocprofv3 --kernel-trace --stats -d $OUT/inferstats -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 13 --warmup 2
step train3 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
grep "^{" $OUT/train3.log | tail -1
step train3s 500 rocprofv3 --kernel-trace --stats -d $OUT/train3s -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
echo all-ok
