#!/bin/bash
# Round 6, the 8-GPU preparation lines on one GPU (verdict task 8) and the
# training step: the config-5 1/8 ray shard through the network (rank 0's
# 512 rays, no collective), with kernel stats; the ddp-train line (N = 1)
# with its Adam roofline; training kernel stats at configs 3 and 4.
set -u
OUT=gpurun_out/${1:-r6b}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
if [ "${TESTS:-}" != "" ]; then
  step tests 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
  tail -2 $OUT/tests.log
fi
L=tools/_lib
step xab_c2 300 python tools/xbench_exact.py "r5=$L/libab_r5.so,hold=$L/libab_hold.so,nt=$L/libab_nt.so" --rounds 5 --iters 10
grep "^{" $OUT/xab_c2.log
step xab_c5 400 python tools/xbench_exact.py "r5=$L/libab_r5.so,hold=$L/libab_hold.so,nt=$L/libab_nt.so" --workload c5_simu_4096x512x2048 --shard-of 8 --rounds 4 --iters 5
grep "^{" $OUT/xab_c5.log
step sigma 300 env AVR_AB_LIB=avr_amd/libavr_hip.so python tools/probe_sigma.py --variant 2 --dtype fp16 --cfgs 0,1,3,6,7,8,0
cat $OUT/sigma.log | grep "^{"
step sigma0 300 env AVR_AB_LIB=avr_amd/libavr_hip.so python tools/probe_sigma.py --variant 0 --dtype fp16 --cfgs 0,1,2,3,0
cat $OUT/sigma0.log | grep "^{"
step c5shard 500 rocprofv3 --kernel-trace --stats -d $OUT/c5shard -o run --output-format csv -- python bench.py --mode ray-shard --network --mlp-dtype fp16 --shard-of 8 --steps 10 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5shard.log | tail -1 > $OUT/c5shard.json
step ddp 500 python bench.py --mode ddp-train --steps 20 --warmup 5
grep "^{" $OUT/ddp.log | tail -1 > $OUT/ddp.json
step train3 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
grep "^{" $OUT/train3.log | tail -1
step train3s 500 rocprofv3 --kernel-trace --stats -d $OUT/train3s -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
grep "^{" $OUT/train3s.log | tail -1
step train4 500 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu --steps 20
grep "^{" $OUT/train4.log | tail -1
echo all-ok
