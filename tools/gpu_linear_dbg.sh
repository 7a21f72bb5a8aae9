#!/bin/bash
# hidden-layer GEMM A/B in one process (200 warm-up pairs): AVR_LINEAR_DBG values (4: nt x stream) interleaved
# with hipBLASLt, several repetitions
set -u
OUT=gpurun_out/linear
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/probe_linear.py --dtype fp16 --dbgs ${DBGS:-0,4} --reps 5 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
grep '^{' $OUT/ab.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d.get('kernel', 'agree'), d.get('dbg', ''), round(d['us'], 1) if 'us' in d else d)
"
