"""Per-item analysis of the exact head's probe records (tools/probe_phases.py
with AVR_PROBE_DUMP): prologue cycles, cycles per tile and their phases,
per-workgroup span.  python tools/exact_items.py DIR"""
import glob
import os
import sys

import numpy as np


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "exact_skip*.npy"))):
        w = np.load(f).astype(np.float64)
        rt0, t1, t2, t3, dma, bar, comp, rt1 = w[:, :8].T
        marks = w[:, 8:12]
        tiles = w[:, 12]
        clk = (t3 - t1).sum() / ((rt1 - rt0).sum() / 100e6)
        life, pro = t3 - t1, t2 - t1
        m = tiles > 0
        mk = [float(np.mean((marks[m, k] - t1[m])[marks[m, k] > 0])) if (marks[m, k] > 0).any() else 0 for k in range(3)]
        print(f"{os.path.basename(f)}: span {(rt1.max() - rt0.min()) / 100:.1f} us, clock {clk / 1e9:.2f} GHz, "
              f"tiles/item {tiles[m].mean():.1f}, prologue {pro[m].mean():.0f} cyc (marks 8/9/10 at "
              f"{mk[0]:.0f}/{mk[1]:.0f}/{mk[2]:.0f}), per tile: body {np.mean((life - pro)[m] / tiles[m]):.0f} "
              f"comp {np.mean(comp[m] / tiles[m]):.0f} dma {np.mean(dma[m] / tiles[m]):.0f} "
              f"bar {np.mean(bar[m] / tiles[m]):.0f} cyc")


if __name__ == "__main__":
    main(sys.argv[1])
