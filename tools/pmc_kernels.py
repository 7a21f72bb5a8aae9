"""Per-kernel medians of the counters of tools/pmc_infer.sh's passes, with
derived figures (MFMA busy, LDS bank-conflict share, L2 hit rate, HBM bytes
with the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md §HBM).

    python tools/pmc_kernels.py <dir with p0..p4> [out.json]
"""
import csv
import glob
import json
import os
import statistics
import sys

KEYS = ("hashgrid_fwd_lm", "sigma_meshrir_h1", "head_exact_kernel", "Cijk", "ray_reduce", "dft_phase", "linear512",
        "linear_xs", "hashgrid")


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:90]


def main(d, out=None):
    data = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not any(x in k for x in KEYS):
                continue
            data.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res = {}
    for k, cs in data.items():
        m = {c: statistics.median(v) for c, v in cs.items()}
        der = {}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            # cycles = 32 x MFMAs (32x32x16) summed over SIMDs: divide by
            # 1024 SIMDs x the launch's cycles for the utilisation
            der["mfma_busy_simd_cycles"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024
        if m.get("SQ_LDS_IDX_ACTIVE"):
            der["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("SQ_WAVE_CYCLES"):
            der["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
        if m.get("TCC_REQ_sum"):
            der["l2_hit_frac"] = m.get("TCC_HIT_sum", 0) / max(1.0, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0))
        if "FETCH_SIZE" in m:
            der["hbm_read_bytes"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            der["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        res[k] = {"counters": m, "derived": {a: b for a, b in der.items() if b is not None}}
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
