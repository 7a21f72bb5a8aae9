#!/bin/bash
# Band-form linear head: partial check, head tests, probe timing and
# kernel stats at config 2.  Stops at the first failing step.
set -u
OUT=gpurun_out/band
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step z 200 python tools/probe_band_z.py --case raf --dtype bf16 --cols 4 --forms 1,0
grep -c '"n_bad": 0' $OUT/z.log
step tests 600 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 120 --timeout-method thread -k "band or linear or config2"
tail -1 $OUT/tests.log
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python tools/probe_band.py --dtype fp16
grep render_ms $OUT/prof.log
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/band/prof/run_kernel_stats.csv')):
    if 'head' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000, 1), round(float(r['MinNs'])/1000, 1))
PY
echo all-ok
