"""Average duration of each consecutive group of head_band_fwd launches in a
rocprofv3 kernel trace (one group per probe_band.py setting, in order)."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "head_band_fwd" in r["Kernel_Name"]]
labels = sys.argv[2].split(",")
per = len(rows) // len(labels)
for i, lab in enumerate(labels):
    g = rows[i * per:(i + 1) * per][3:]  # skip the warm-up launches
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in g]
    print(f"dbg {lab}: {sum(d) / len(d) / 1000:.1f} us over {len(d)} launches")
