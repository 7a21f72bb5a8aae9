"""A/B timing of the fused sigma kernel (`avr_sigma_fwd`) across library
builds and tile configs at config-2 size, interleaved in one process (HIP
events); outputs compared bitwise with the first entry's.

    python tools/xbench_sigma.py old=tools/_lib/libab_sig_old.so:identity:0 \\
        cur=avr_amd/libavr_hip.so:stream:0,9,10,11 [--variant 2] [--dtype fp16]

Each entry is name=library:pack order:tile configs; "identity" packs the
layers in SCHEDULE order (builds before sigma.STREAM_ORDER), "stream" in the
current stream order.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import _lib, sigma  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("entries", nargs="+")
    ap.add_argument("--variant", type=int, default=sigma.MESHRIR_H1)
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="fp16", choices=["bf16", "fp16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    v = a.variant
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    ws = [torch.randn(M, K, device=dev, generator=g) * np.sqrt(2.0 / K) for M, K, _, _ in sigma.SCHEDULE[v]]
    N, S = a.n, 256
    inputs = [(torch.rand(N, 40, device=dev, generator=g).half(), 1)]
    bias = torch.randn(-(-N // S), 512, device=dev, generator=g) * 0.1 if v == sigma.MESHRIR_H1 else None
    out_w = 512 if v == sigma.MESHRIR_H1 else 128
    extras = [] if v == sigma.MESHRIR_H1 else [(torch.rand(N // S, 40, device=dev, generator=g).half(), S),
                                               (torch.rand(1, 40, device=dev, generator=g).half(), N)]
    flops = 2 * N * sum(M * K for M, K, _, _ in sigma.SCHEDULE[v])
    runs = []
    saved = sigma.STREAM_ORDER
    for e in a.entries:
        name, rest = e.split("=", 1)
        path, order, cfgs = rest.split(":")
        lib = ctypes.CDLL(path if os.path.isabs(path) else os.path.join(ROOT, path))
        lib.avr_sigma_fwd.restype, lib.avr_sigma_fwd.argtypes = _lib._SIGS["avr_sigma_fwd"]
        lib.avr_last_error.restype = ctypes.c_char_p
        sigma.STREAM_ORDER = saved if order == "stream" else {}
        packed = sigma.pack_layers(v, ws, dt)
        sigma.STREAM_ORDER = saved
        for c in cfgs.split(","):
            runs.append((f"{name}/{c}", lib, packed, int(c)))
    results = {k: [] for k, *_ in runs}
    outs = {}
    for rnd in range(a.rounds):
        for key, lib, packed, cfg in runs:
            _lib._lib = lib  # route sigma_fwd's call to this build

            def launch():
                return sigma.sigma_fwd(v, packed, N, inputs, extras, out_w, 0.01, tile_cfg=cfg, bias=bias,
                                       bias_div=S)

            for _ in range(5):
                out = launch()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                out = launch()
            e1.record()
            torch.cuda.synchronize()
            results[key].append(e0.elapsed_time(e1) * 1e3 / a.iters)
            if rnd == 0:
                outs[key] = out
    first = runs[0][0]
    for key in results:
        us = min(results[key])
        same = all(torch.equal(x, y) for x, y in zip(outs[key], outs[first]))
        print(json.dumps({"variant": v, "dtype": a.dtype, "entry": key, "n": N, "us_min": us,
                          "us_all": [round(t, 2) for t in results[key]], "tflops": flops / (us * 1e-6) / 1e12,
                          "bitwise_equal_to_first": same}))


if __name__ == "__main__":
    main()
