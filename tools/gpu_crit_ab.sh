#!/bin/bash
# Loss total: criterion kernel vs seven torch adds, config-3 and config-4
# training steps alternated three times in one box.
set -u
OUT=gpurun_out/${1:-critab}
mkdir -p $OUT
for i in 1 2 3; do
  for v in kernel torch; do
    flag=""; [ $v = torch ] && flag="--torch-total"
    for w in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
      timeout -k 10 300 python tools/bench_train.py --workload $w --steps 40 $flag > $OUT/${v}_${w}_$i.log 2>&1 || { echo "$v $w rc=$?"; tail -20 $OUT/${v}_${w}_$i.log; exit 1; }
      echo "$v $w $i $(grep -o '"train_step_ms": [0-9.]*' $OUT/${v}_${w}_$i.log)"
    done
  done
done
echo all-ok
