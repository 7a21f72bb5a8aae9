"""GPU probe: the linear fused head's forward, band form (csrc/head_band.hip)
against the feature-block form (head_fwd_kernel, AVR_HEAD_BAND=0), at a
workload's shape: render time through render_from_hidden (no autograd), and
the relative difference of the two spectra.  Kernel times come from running
it under rocprofv3 --kernel-trace --stats.

    python tools/probe_band.py [--workload c2_meshrir_1024x256x512] [--K 512] [--dtype fp16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--forms", default="1,0")
    ap.add_argument("--dbgs", default="0", help="AVR_HEAD_BAND_DBG values (timing experiments)")
    ap.add_argument("--reps", type=int, default=1, help="repetitions of the whole set, interleaved")
    ap.add_argument("--warmup", type=int, default=0, help="untimed renders of each form before any timing")
    ap.add_argument("--bufs", default="4", help="AVR_HEAD_BAND_BUF values for the band form")
    args = ap.parse_args()
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, args.K
    r = AVRRender(None, exact_head=False, **w.render)
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    _, _, _, _, geom = r.sample(ro, tx)
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(dt)
    W = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
    outs = {}
    with torch.no_grad():
        runs = [(f, rg, d) for f in args.forms.split(",") for rg in (args.bufs.split(",") if f == "1" else ["4"])
                for d in (args.dbgs.split(",") if f == "1" else ["0"])] * args.reps
        for _ in range(args.warmup):  # clocks up before anything is timed
            for f in args.forms.split(","):
                os.environ["AVR_HEAD_BAND"] = f
                r.render_from_hidden(attn, h, W, dt, geom)
        torch.cuda.synchronize()
        for form, ring, dbg in runs:
            os.environ["AVR_HEAD_BAND"] = form
            os.environ["AVR_HEAD_BAND_BUF"] = ring
            os.environ["AVR_HEAD_BAND_DBG"] = dbg
            for _ in range(3):
                out = r.render_from_hidden(attn, h, W, dt, geom)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                r.render_from_hidden(attn, h, W, dt, geom)
            e1.record()
            e1.synchronize()
            if dbg == "0":
                outs[form] = out.double().cpu()
            print(json.dumps({"workload": w.name, "K": K, "dtype": args.dtype, "band": int(form), "chunk_slots": int(ring), "dbg": int(dbg),
                              "render_ms": e0.elapsed_time(e1) / args.iters}), flush=True)
    os.environ.pop("AVR_HEAD_BAND", None)
    if "1" in outs and "0" in outs:
        a, b = outs["1"], outs["0"]
        print(json.dumps({"band_vs_blocks_rel_l2": float((a - b).norm() / b.norm()),
                          "band_vs_blocks_rel_max": float((a - b).abs().max() / b.abs().max())}), flush=True)


if __name__ == "__main__":
    main()
