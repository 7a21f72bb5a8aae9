"""GPU probe: work balance of the persistent exact head (head_exact.hip,
AVR_HEAD_EXACT_WAVES 19) at config 2, from the delay sort of random poses.

Model: a workgroup's time is the sum over its columns of the 64-ray tiles it
runs, ceil(cnt[last live t of its t-block] / 64).  Static assignment (the
kernel's): XCD x owns columns [x*cpx, (x+1)*cpx), workgroup m of the XCD
keeps t-block m % ntb and walks columns x*cpx + m/ntb + k*(wg/ntb).  Printed:
the max over workgroups against the mean (the ideal balance), per pose.

    python tools/probe_exact_balance.py [--poses 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, _lib  # noqa: E402
from avr_amd import renderer as rd  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=8)
    ap.add_argument("--wg", type=int, default=32, help="workgroups per XCD")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    B, R, S, T = 1, w.n_rays, w.n_samples, w.T
    r = AVRRender(None, **w.render)
    g = torch.Generator(device=dev).manual_seed(0)
    TB, ntb = 256, (T + 255) // 256
    ncol = B * S
    cpx = (ncol + 7) // 8
    nq = args.wg // ntb
    for i in range(args.poses):
        ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
        tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
        _, _, _, _, geom = r.sample(ro, tx)
        attn = torch.rand(B, R * S, device=dev, generator=g) * 2
        p = r._params(T, R)
        tables = rd.get_tables(p, dev)
        st = rd._stream(dev)
        pref = rd.ctypes_ref(p)
        wts, delay = rd._weights(p, attn, geom["rays_o"], geom["position_tx"], geom["dirs"], tables, st)
        perm = torch.empty(B, S, R, dtype=torch.int32, device=dev)
        ws = torch.empty(B, S, R, dtype=torch.float32, device=dev)
        cnt = torch.empty(B, S, T, dtype=torch.int32, device=dev)
        _lib.call("avr_head_sort", pref, B, rd._ptr(wts), rd._ptr(delay), rd._ptr(perm), rd._ptr(ws),
                  rd._ptr(cnt), st)
        torch.cuda.synchronize()
        c = cnt[0].long().cpu()
        lim = (T - 1 - tables.shift.long().cpu()).clamp(max=T)
        # tiles[col][tb]
        tiles = torch.zeros(ncol, ntb)
        for s in range(S):
            for tb in range(ntb):
                tl = min(tb * TB + TB, int(lim[s])) - 1
                if tl >= tb * TB:
                    tiles[s, tb] = (int(c[s, tl]) + 63) // 64
        wg_work = []
        for x in range(8):
            for m in range(args.wg):
                tb = m % ntb
                cols = range(x * cpx + m // ntb, min(ncol, (x + 1) * cpx), nq)
                wg_work.append(float(sum(tiles[cc, tb] for cc in cols)))
        per_tb = tiles.sum(0).tolist()
        mx, mean = max(wg_work), sum(wg_work) / len(wg_work)
        print(json.dumps({"pose": i, "max_wg_tiles": mx, "mean_wg_tiles": round(mean, 1),
                          "balance": round(mean / mx, 3), "tiles_per_tblock": per_tb}), flush=True)


if __name__ == "__main__":
    main()
