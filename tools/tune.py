"""GPU tuning sweep (run on the box): reduction variant x n_split x k_split
x column group G for one workload, interleaved rounds in one
process (cdna guide §5.4 rule 24), cycling over --poses synthetic poses.

    python tools/tune.py [--workload c2_meshrir_1024x256x512] [--rounds 5]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, spectrum_to_ir  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402
from bench import KernelTimer, StubNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--variants", default="u4nt,u8nt")
    ap.add_argument("--nsplit", default="1,2,4")
    ap.add_argument("--ksplit", default="4,8,16")
    ap.add_argument("--T", type=int, default=0)
    ap.add_argument("--S", type=int, default=0)
    ap.add_argument("--nazi", type=int, default=0)
    ap.add_argument("--dtype", default="")
    ap.add_argument("--G", default="", help="AVR_REDUCE_G values, e.g. 1,2 (default: library rule)")
    ap.add_argument("--poses", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    over = {}
    if args.T:
        over["T"] = args.T
    if args.S:
        over["n_samples"] = args.S
    if args.nazi:
        over["n_azi"] = args.nazi
    if args.dtype:
        over["signal_dtype"] = args.dtype
        over["attn_dtype"] = args.dtype
    if over:
        w = w.replace(**over)
    print(json.dumps({"workload": w.name, "R": w.n_rays, "S": w.n_samples, "T": w.T,
                      "dtype": w.signal_dtype}))
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    dt = torch.float16 if w.signal_dtype == "float16" else torch.float32
    g = torch.Generator(device=dev).manual_seed(0)
    attn = (torch.rand(B, R * S, 1, device=dev, generator=g) * 2).to(dt)
    sig = (torch.randn(B, R * S, T, device=dev, generator=g) * 0.1).to(dt)
    P = max(1, args.poses)
    ro = torch.rand(P, B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(P, B, 3, device=dev, generator=g) * 4 - 2
    dtx = (torch.nn.functional.normalize(torch.randn(P, B, 3, device=dev, generator=g), dim=-1)
           if w.with_dir_tx else [None] * P)
    r = AVRRender(StubNet(attn, sig), **w.render)
    timer = KernelTimer(args.steps)
    r.kernel_timer = timer
    opt = lambda a: a.split(",") if a else [""]  # noqa: E731
    combos = list(itertools.product(args.variants.split(","), [int(x) for x in args.nsplit.split(",")],
                                    [int(x) for x in args.ksplit.split(",")], opt(args.G)))
    res = {c: {"step": [], "reduce": []} for c in combos}
    es = 2 if dt == torch.float16 else 4
    for rnd in range(args.rounds):
        for c in combos:
            v, ns, ks, gg = c
            if gg:
                os.environ["AVR_REDUCE_G"] = gg
            else:
                os.environ.pop("AVR_REDUCE_G", None)
            os.environ["AVR_REDUCE_VARIANT"] = v
            os.environ["AVR_NSPLIT"] = str(ns)
            if ks:
                os.environ["AVR_KSPLIT"] = str(ks)
            else:
                os.environ.pop("AVR_KSPLIT", None)
            with torch.no_grad():
                for i in range(3):
                    spectrum_to_ir(r(ro[i % P], tx[i % P], dtx[i % P]))
                torch.cuda.synchronize()
                timer.used = 0
                timer.rows.clear()
                timer.enabled = True
                t0 = time.perf_counter()
                for i in range(args.steps):
                    spectrum_to_ir(r(ro[i % P], tx[i % P], dtx[i % P]))
                torch.cuda.synchronize()
                dt_s = (time.perf_counter() - t0) / args.steps
                timer.enabled = False
            res[c]["step"].append(dt_s * 1e3)
            res[c]["reduce"].append(timer.mean_ms())
    out = []
    for c, d in res.items():
        v, ns, ks, gg = c
        red = statistics.median(d["reduce"])
        byts = w.ray_samples * (T * es + 8) + ns * B * S * T * 4
        out.append(dict(variant=v, n_split=ns, k_split=ks, G=gg, step_ms=statistics.median(d["step"]),
                        step_min=min(d["step"]), reduce_ms=red, reduce_gbs=byts / red / 1e6))
    out.sort(key=lambda x: x["step_ms"])
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
