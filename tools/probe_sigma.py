"""Time the fused sigma kernel (csrc/sigma.hip) per tile config at config-2
size (262144 samples) with HIP events; prints one JSON line per config.

    python tools/probe_sigma.py [--variant 0|1] [--n 262144] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from avr_amd import _lib, sigma  # noqa: E402

# tile configs >= 16 (timing experiments, garbage results) exist only in the
# shapes build: make -C avr_amd/csrc shapes
_lib.LIB_PATH = os.environ.get("AVR_AB_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "_lib", "libavr_shapes.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cfgs", default="0,1,2")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    v = a.variant
    ws = [torch.randn(M, K, device=dev) * np.sqrt(2.0 / K) for M, K, _, _ in sigma.SCHEDULE[v]]
    packed = sigma.pack_layers(v, ws, torch.float16 if a.dtype == "fp16" else torch.bfloat16)
    N, S, RS = a.n, 256, 262144
    B = -(-N // RS)
    bias = None
    if v == sigma.MESHRIR_H1:
        inputs = [(torch.rand(N, 40, device=dev).half(), 1)]
        extras = []
        out_w = 512
        bias = torch.randn(-(-N // S), 512, device=dev) * 0.1
    elif v == sigma.MESHRIR:
        inputs = [(torch.rand(N, 40, device=dev).half(), 1)]
        extras = [(torch.rand(B * RS // S, 40, device=dev).half(), S), (torch.rand(B, 40, device=dev).half(), RS)]
        out_w = 128
    else:
        inputs = [(torch.rand(N, 40, device=dev), 1), (torch.rand(B, 40, device=dev), RS)]
        extras = [(torch.rand(B * RS // S, 40, device=dev), S), (torch.rand(B, 40, device=dev), RS),
                  (torch.rand(N, 40, device=dev), 1), (torch.rand(B, 40, device=dev), RS)]
        out_w = 256
    flops = 2 * N * sum(M * K for M, K, _, _ in sigma.SCHEDULE[v])
    for cfg in [int(c) for c in a.cfgs.split(",")]:
        import time
        t_end = time.time() + 0.5  # clocks settle before timing
        while time.time() < t_end:
            for _ in range(20):
                sigma.sigma_fwd(v, packed, N, inputs, extras, out_w, 0.01, tile_cfg=cfg, bias=bias, bias_div=S)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            sigma.sigma_fwd(v, packed, N, inputs, extras, out_w, 0.01, tile_cfg=cfg, bias=bias, bias_div=S)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(json.dumps({"variant": v, "dtype": a.dtype, "tile_cfg": cfg, "n": N, "us": us,
                          "tflops": flops / (us * 1e-6) / 1e12}))


if __name__ == "__main__":
    main()
