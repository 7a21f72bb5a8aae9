"""Average rocprofv3 --pmc counters per kernel over dispatches:
python tools/pmc_read.py <dir> [<dir> ...] [--match substr]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = ""
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args = [a for a in args if a != match]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"]:
                continue
            agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
