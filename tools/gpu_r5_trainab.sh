#!/bin/bash
# Training-step A/B (configs 3 and 4): the shipped defaults against one
# switch at a time (env assignments given as arguments, e.g. AVR_TUNABLEOP=0),
# after one throwaway process (a fresh box's first run is slower), each pair
# run twice, interleaved.
set -u
OUT=gpurun_out/${TAG:-trainab}
mkdir -p $OUT
run() {  # workload, label, env...
  local wl=$1 lab=$2; shift 2
  env "$@" timeout -k 10 200 python tools/bench_train.py --workload $wl --steps ${STEPS:-40} > $OUT/${wl}_$lab.log 2>&1 || { tail -20 $OUT/${wl}_$lab.log; exit 1; }
  tail -1 $OUT/${wl}_$lab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl $lab', round(d['train_step_ms'],3))"
}
run c3_raf_furnished_b4 warm X=0
for wl in c3_raf_furnished_b4 c4_raf_empty_b4_per_gpu; do
  for rep in 1 2; do
    run $wl default_$rep X=0
    for sw in "$@"; do run $wl ${sw}_$rep $sw; done
  done
done
