"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel
HBM bytes per launch (profiles/*.json), applying the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a wide
coalesced streaming read (x2), WRITE_SIZE is exact for 16-B stores; both are
in KiB.

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write out.json [workload]
"""
from __future__ import annotations

import csv
import json
import os
import re
import statistics
import sys


def per_kernel(path):
    rows = list(csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))))
    by = {}
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        by.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: (statistics.median(v), len(v)) for k, v in by.items()}


def main(fetch_dir, write_dir, out, workload="c2_meshrir_1024x256x512"):
    f = per_kernel(fetch_dir)
    w = per_kernel(write_dir)
    import datetime
    m = re.match(r"r(\d+)_", os.path.basename(out))
    res = {"workload": workload, "unit": "bytes per launch",
           # bench.py's pmc_traffic takes the newest summary by (round, measured_at)
           "round": int(m.group(1)) if m else 0,
           "measured_at": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds"),
           "correction": "FETCH_SIZE*1024*2 (gfx950 half-count on wide streaming reads), WRITE_SIZE*1024",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fk = f.get(k, (0.0, 0))[0]
        wk = w.get(k, (0.0, 0))[0]
        res["kernels"][k] = {"fetch_kib_raw": fk, "write_kib_raw": wk,
                             "hbm_read_bytes": fk * 1024 * 2, "hbm_write_bytes": wk * 1024,
                             "hbm_bytes": fk * 1024 * 2 + wk * 1024, "launches": f.get(k, (0, 0))[1]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
