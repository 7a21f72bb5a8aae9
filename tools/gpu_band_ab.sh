#!/bin/bash
# Band head against the feature-block head, warmed up and interleaved in one
# process (render_from_hidden at config 2), under rocprofv3 kernel trace.
set -u
OUT=gpurun_out/band
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/ab -o run --output-format csv -- python tools/probe_band.py --dtype ${DT:-fp16} --forms 1,0 --bufs 4,3 --reps 4 --warmup 100 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
grep render_ms $OUT/ab.log | cut -c1-140
python - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/band/ab/run_kernel_trace.csv')))
for key in ("head_band_fwd_kernel<__half>", "head_band_fwd_kernel<__half, 3>", "head_fwd_kernel"):
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if key in r["Kernel_Name"]]
    if not d:
        continue
    d = d[len(d) // 2:]  # second half: after the warm-up
    print(key, round(sum(d) / len(d) / 1000, 1), "us over", len(d))
PY
