#!/bin/bash
# Round-5 final: every GPU test, smoke(), the driver's bench command, kernel
# stats of config-2 fp16 inference and of the config-5 ray-shard line through
# the reference network, and the inference counter passes.
set -u
OUT=gpurun_out/${1:-r5final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
  tail -2 $OUT/tests.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $OUT/smoke.log
fi
step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5
tail -1 $OUT/bench.log > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'], d['network_inference']['ms_per_pose'])"
step inferstats 400 rocprofv3 --kernel-trace --stats -d $OUT/infer -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 13 --warmup 2
grep "^{" $OUT/inferstats.log | tail -1
step c5net 500 rocprofv3 --kernel-trace --stats -d $OUT/c5net -o run --output-format csv -- python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5net.log | tail -1 > $OUT/c5net.json
step pmc 900 bash tools/pmc_infer.sh $OUT/pmc
tail -30 $OUT/pmc.log
echo all-ok
