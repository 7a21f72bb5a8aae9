#!/bin/bash
# Round-5 evidence for the bench line's roofline: kernel stats of the
# driver's bench command, and the two PMC passes (separate runs, no trace
# domains) summarised into HBM bytes per launch (tools/pmc_summary.py).
set -u
OUT=gpurun_out/${1:-r5benchprof}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -30 $OUT/$name.log; exit $rc; fi
  echo "$name ok"
}
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
grep "^{" $OUT/stats.log | tail -1 > $OUT/stats_bench.json
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --no-network --steps 20 --warmup 3 --streams 1
python tools/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/r05_pmc_c2_end.json c2_meshrir_1024x256x512 && echo summary-ok
