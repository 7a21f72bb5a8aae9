# Per-kernel breakdown of the fused config-2 inference pose (bf16 and fp16).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for dt in bf16 fp16; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ip_$dt -o run --output-format csv -- python tools/bench_infer.py --variants fused --steps 20 --warmup 3 --mlp-dtype $dt > gpurun_out/ip_$dt.log 2>&1 || exit 1
tail -1 gpurun_out/ip_$dt.log
python - $dt <<'PY'
import csv, sys
dt = sys.argv[1]
rows = list(csv.DictReader(open(f'gpurun_out/ip_{dt}/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:22]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs'])/1000:8.2f} {float(r['TotalDurationNs'])/tot*100:5.1f}%")
PY
done
