#!/bin/bash
# Round-4 validation and the profiles it commits: every GPU test, smoke(),
# the driver's bench command twice, kernel stats of the pipelined bench and of
# a single-stream (--streams 1) run, the FETCH_SIZE / WRITE_SIZE passes of the
# ray reduction, kernel stats of config-2 fp16 inference and the config-3
# training step, the network ray-shard line.
set -u
OUT=gpurun_out/${1:-r4val}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -W ignore
tail -2 $OUT/tests.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $OUT/smoke.log
for i in 1 2; do
  step bench$i 400 python bench.py --gpus 1 --steps 20 --warmup 5
  tail -1 $OUT/bench$i.log > $OUT/bench$i.json
  python -c "import json; d=json.load(open('$OUT/bench$i.json')); print('bench', d['value'], d['ms_per_step'], d['ms_per_step_graph'], d['ir_render_ms_per_pose'], d['roofline']['avg_launch_ms'], d['network_inference']['ms_per_pose'])"
done
step prof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline
step prof1 400 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline --streams 1
grep "^{" $OUT/prof1.log | tail -1 > $OUT/prof1.json
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1
step profinfer 400 rocprofv3 --kernel-trace --stats -d $OUT/profinfer -o run --output-format csv -- python tools/bench_infer.py --mlp-dtype fp16 --variants fused --steps 10 --warmup 3
tail -3 $OUT/profinfer.log
step proftrain 400 rocprofv3 --kernel-trace --stats -d $OUT/proftrain -o run --output-format csv -- python tools/bench_train.py --steps 5 --warmup 2
step rayshard_net 400 python bench.py --mode ray-shard --network --mlp-dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline
tail -1 $OUT/rayshard_net.log
echo all-ok
