#!/bin/bash
# Round 6 end-of-round evidence: every GPU test, smoke(), the driver's bench
# command, its kernel stats and the two PMC passes of the ray reduction,
# config-2 fp16 inference kernel stats, the config-5 1/8 ray-shard line and
# the ddp-train line, the training step at configs 3 and 4.
set -u
OUT=gpurun_out/${1:-r6final}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -1 $OUT/tests.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/smoke.log
step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5
tail -1 $OUT/bench.log > $OUT/bench.json
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --streams 1
grep "^{" $OUT/stats.log | tail -1 > $OUT/stats_bench.json
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1
python tools/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/r06_pmc_c2_final.json c2_meshrir_1024x256x512 > $OUT/pmc_summary.log && echo summary-ok
step infer 400 rocprofv3 --kernel-trace --stats -d $OUT/infer -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 13 --warmup 2
step c5shard 500 rocprofv3 --kernel-trace --stats -d $OUT/c5shard -o run --output-format csv -- python bench.py --mode ray-shard --network --mlp-dtype fp16 --shard-of 8 --steps 10 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5shard.log | tail -1 > $OUT/c5shard.json
step c5shard_plain 400 python bench.py --mode ray-shard --network --mlp-dtype fp16 --shard-of 8 --steps 10 --warmup 2
grep "^{" $OUT/c5shard_plain.log | tail -1 > $OUT/c5shard_plain.json
step c5net 500 python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
grep "^{" $OUT/c5net.log | tail -1 > $OUT/c5net.json
step ddp 500 python bench.py --mode ddp-train --steps 20 --warmup 5
grep "^{" $OUT/ddp.log | tail -1 > $OUT/ddp.json
step train3 300 python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 30
grep "^{" $OUT/train3.log | tail -1
step train3s 500 rocprofv3 --kernel-trace --stats -d $OUT/train3s -o run --output-format csv -- python tools/bench_train.py --workload c3_raf_furnished_b4 --steps 20
step train4 500 python tools/bench_train.py --workload c4_raf_empty_b4_per_gpu --steps 20
grep "^{" $OUT/train4.log | tail -1
echo all-ok
