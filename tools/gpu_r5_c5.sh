#!/bin/bash
set -u
OUT=gpurun_out/${1:-r5c5}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 900 python -u -m pytest tests/test_tunableop.py tests/test_gpu_head.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -2 $OUT/tests.log
step c5net 500 rocprofv3 --kernel-trace --stats -d $OUT/c5net -o run --output-format csv -- python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5net.log | tail -1 > $OUT/c5net.json
cat $OUT/c5net.json | cut -c1-300
step c5plain 500 python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5plain.log | tail -1 | cut -c1-300
echo all-ok
