#!/bin/bash
# Round 6 GPU check: GPU tests (TESTS= to narrow), smoke, the driver's bench
# command, kernel stats of config-2 fp16 inference and of the config-3
# training step.  Every step under its own time limit; the first failure ends
# the call.
set -u
OUT=gpurun_out/${1:-r6}
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
  step tests ${TEST_SECS:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
  tail -2 $OUT/tests.log
fi
if [ "${SKIP_SMOKE:-0}" != 1 ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $OUT/smoke.log
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5
  tail -1 $OUT/bench.log > $OUT/bench.json
  python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'], d['network_inference']['ms_per_pose'])"
fi
if [ "${SKIP_INFER:-0}" != 1 ]; then
  step inferstats 400 rocprofv3 --kernel-trace --stats -d $OUT/infer -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 13 --warmup 2
  grep "^{" $OUT/inferstats.log | tail -1
fi
if [ "${SKIP_TRAIN:-0}" != 1 ]; then
  step trainstats 500 rocprofv3 --kernel-trace --stats -d $OUT/train -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
  grep "^{" $OUT/trainstats.log | tail -1
fi
echo all-ok
