#!/bin/bash
# XCD-aware DFT order: render/graph/head tests, the driver's bench command,
# kernel stats + PMC FETCH_SIZE of the DFT.
set -u
OUT=gpurun_out/dftx
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -W ignore tests/test_gpu_render.py tests/test_gpu_graph.py tests/test_gpu_head.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  tail -1 $OUT/b$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], d['ms_per_step_eager'], d['ir_render_ms_per_pose'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-network --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1 > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python - <<'PY'
import csv, glob, statistics
f = glob.glob('gpurun_out/dftx/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'dft_phase_fwd' in r['Name'] or 'ray_reduce_fwd' in r['Name']:
        print(r['Name'][:50], r['Calls'], r['AverageNs'])
f = glob.glob('gpurun_out/dftx/pmc/**/*counter_collection.csv', recursive=True)[0]
v = [float(r['Counter_Value']) for r in csv.DictReader(open(f)) if 'dft_phase_fwd' in r['Kernel_Name']]
print('dft FETCH_SIZE KiB median', statistics.median(v), 'x2 bytes', statistics.median(v) * 2048)
PY
