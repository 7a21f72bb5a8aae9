#!/bin/bash
# Round-5 late check: every GPU test, smoke(), the driver's bench command,
# then the training A/B of the narrow-layer switch.
set -u
OUT=gpurun_out/${1:-r5check3}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -2 $OUT/tests.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/smoke.log
step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5
tail -1 $OUT/bench.log > $OUT/bench.json
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'], d['network_inference']['ms_per_pose'])"
TAG=$(basename $OUT)_ab STEPS=40 bash tools/gpu_r5_trainab.sh AVR_NARROW=0
echo all-ok
