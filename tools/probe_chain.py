"""Time the signal network's two 512 -> 512 ReLU layers at config 2
(262144 samples, fp16) as two whole-batch hipBLASLt GEMMs against the same
GEMMs over row chunks, each chunk's intermediate activation reused from a
small buffer (it stays in the Infinity Cache / L2 instead of making an HBM
round trip); outputs must be bit-identical.

    python tools/probe_chain.py [--chunks 131072,65536,32768,16384]
"""
from __future__ import annotations

import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--chunks", default="131072,65536,32768,16384")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(a.n, 512, device=dev, generator=g).to(dt)
    w2 = (torch.randn(512, 512, device=dev, generator=g) * 0.05).to(dt)
    w3 = (torch.randn(512, 512, device=dev, generator=g) * 0.05).to(dt)
    z = torch.zeros(512, device=dev, dtype=dt)
    w2t, w3t = w2.t(), w3.t()

    def full():
        y2 = torch._addmm_activation(z, x, w2t, use_gelu=False)
        return torch._addmm_activation(z, y2, w3t, use_gelu=False)

    y_ref = full()
    out = torch.empty_like(y_ref)

    def chunked(c):
        tmp = torch.empty(c, 512, device=dev, dtype=dt)

        def run():
            for r0 in range(0, a.n, c):
                r1 = min(a.n, r0 + c)
                t = tmp[: r1 - r0]
                torch._addmm_activation(z, x[r0:r1], w2t, use_gelu=False, out=t)
                torch._addmm_activation(z, t, w3t, use_gelu=False, out=out[r0:r1])
            return out
        return run

    def time_us(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    res = {"n": a.n, "dtype": a.dtype}
    for rnd in range(2):
        res[f"full_us_{rnd}"] = time_us(full)
        for c in [int(v) for v in a.chunks.split(",")]:
            fn = chunked(c)
            res[f"chunk{c}_us_{rnd}"] = time_us(fn)
            if rnd == 0:
                res[f"chunk{c}_equal"] = bool(torch.equal(fn(), y_ref))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
