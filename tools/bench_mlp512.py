"""Two width-512 hidden layers: the fused launch (csrc/mlp512.hip) against
the per-layer hipBLASLt GEMMs the model runs otherwise (with the shipped
TunableOp solution where its shape is listed), HIP events, interleaved.

    python tools/bench_mlp512.py [--rows 262144,2097152] [--dtype fp16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="262144,2097152")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    w1 = torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5
    w2 = torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5
    for M in (int(v) for v in a.rows.split(",")):
        x = torch.relu(torch.randn(M, 512, device=dev, generator=g)).to(dt)

        def fused():
            return model._mlp512x2(x, w1, w2, dt)

        def per_layer():
            h = model._LinearReLU.apply(x, w1, dt, True)
            return model._LinearReLU.apply(h, w2, dt, True)

        with torch.no_grad():
            yf, yp = fused(), per_layer()
            torch.cuda.synchronize()
            diff = float(((yf.float() - yp.float()).abs() / yp.float().abs().clamp(min=1e-2)).max())
            times = {"fused": [], "per_layer": []}
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.iters)]
            for _ in range(a.rounds):
                for name, fn in (("fused", fused), ("per_layer", per_layer)):
                    for e0, e1 in ev:
                        e0.record()
                        fn()
                        e1.record()
                    torch.cuda.synchronize()
                    times[name] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
        res = {"rows": M, "dtype": a.dtype, "max_rel_diff_vs_per_layer": diff}
        for k, v in times.items():
            v.sort()
            res[k + "_median_us"] = v[len(v) // 2]
            res[k + "_min_us"] = v[0]
        flops = 2 * 2 * M * 512 * 512
        res["fused_pflops"] = flops / (res["fused_median_us"] * 1e-6) / 1e15
        res["fused_hbm_tbs"] = 2 * M * 512 * x.element_size() / (res["fused_median_us"] * 1e-6) / 1e12
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
