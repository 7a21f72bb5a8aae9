#!/bin/bash
# Round 6: clip coefficient A/B on one box (torch foreach norm vs
# avr_grad_clip_coef), interleaved, config 3; training tests.
set -u
OUT=gpurun_out/${1:-r6d}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 300 python -u -m pytest tests/test_gpu_training.py -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
for i in 1 2 3; do
  step torch$i 200 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30 --torch-norm
  grep "^{" $OUT/torch$i.log | tail -1 >> $OUT/ab.jsonl
  step native$i 200 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
  grep "^{" $OUT/native$i.log | tail -1 >> $OUT/ab.jsonl
done
python -c "
import json
for l in open('$OUT/ab.jsonl'): d=json.loads(l); print(d.get('train_step_ms'))
"
step stats 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
echo all-ok
