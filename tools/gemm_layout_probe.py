"""GPU probe: operand layouts of the signal network's 512 -> 512 ReLU layer
at config 2 (M = 262144 samples, fp16), i.e. which hipBLASLt solution the
call form selects.  Prints one JSON line per variant (us per call) and the
max difference to the current form.

    python tools/gemm_layout_probe.py [--m 262144] [--dtype fp16]
"""
from __future__ import annotations

import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=262144)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    dt = {"fp16": torch.float16, "bf16": torch.bfloat16}[args.dtype]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(args.m, args.k, device=dev, generator=g) * 0.5).to(dt)
    w = (torch.randn(args.n, args.k, device=dev, generator=g) / args.k ** 0.5).to(dt)
    wt = w.t().contiguous()
    z = torch.zeros(args.n, device=dev, dtype=dt)
    xt = x.t().contiguous()  # a producer could write the transposed layout directly
    variants = {
        "addmm_act_wT_view": lambda: torch._addmm_activation(z, x, w.t(), use_gelu=False),
        "addmm_act_wT_contig": lambda: torch._addmm_activation(z, x, wt, use_gelu=False),
        "mm_then_relu": lambda: torch.relu_(x @ w.t()),
        "mm_wT_contig_then_relu": lambda: torch.relu_(x @ wt),
        "out_transposed": lambda: torch.relu_(w @ xt).t(),
        "out_transposed_xview": lambda: torch.relu_(w @ x.t()).t(),
    }
    ref = variants["addmm_act_wT_view"]().float()
    for name, fn in variants.items():
        y = fn()
        torch.cuda.synchronize()
        diff = float((y.float() - ref).abs().max())
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        flop = 2.0 * args.m * args.n * args.k
        print(json.dumps({"variant": name, "us": us, "tflops": flop / us / 1e6, "max_abs_diff": diff}),
              flush=True)


if __name__ == "__main__":
    main()
