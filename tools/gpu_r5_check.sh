#!/bin/bash
# Round-5 GPU check: every GPU test, smoke(), the driver's bench command, and
# the config-5 ray-shard line through the reference network (AVRModel,
# avr_simu.yml, fp16 MLPs) under rocprofv3 kernel stats.
set -u
OUT=gpurun_out/${1:-r5check}
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
  step tests 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
  tail -2 $OUT/tests.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $OUT/smoke.log
fi
step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5
tail -1 $OUT/bench.log > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'], d['network_inference']['ms_per_pose'])"
step c5net 500 rocprofv3 --kernel-trace --stats -d $OUT/c5net -o run --output-format csv -- python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5net.log | tail -1 > $OUT/c5net.json
echo all-ok
