#!/bin/bash
# Same-box A/B of the training step: this tree against a copy of another
# tree placed under gpu_ab/<name>/ (avr_amd/ with its built library and
# tools/bench_train.py), runs interleaved.
#   bash tools/gpu_trainab.sh OUT NAME [workload]
set -u
OUT=gpurun_out/${1:-trainab}; NAME=${2:-r5}; WL=${3:-c3_raf_furnished_b4}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_train.py --workload $WL --steps 30 > $OUT/cur_$i.log 2>&1 || { echo "cur_$i failed"; tail -20 $OUT/cur_$i.log; exit 1; }
  grep "^{" $OUT/cur_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cur', d['train_step_ms'])"
  (cd gpu_ab/$NAME && timeout -k 10 200 python tools/bench_train.py --workload $WL --steps 30) > $OUT/${NAME}_$i.log 2>&1 || { echo "${NAME}_$i failed"; tail -20 $OUT/${NAME}_$i.log; exit 1; }
  grep "^{" $OUT/${NAME}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$NAME', d['train_step_ms'])"
done
timeout -k 10 200 python tools/host_prof_train.py --workload $WL > $OUT/hostprof_cur.log 2>&1 || { echo hostprof failed; tail -20 $OUT/hostprof_cur.log; exit 1; }
echo all-ok
