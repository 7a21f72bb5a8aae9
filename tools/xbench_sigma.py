"""A/B timing of the fused sigma kernels (`avr_sigma_fwd`, csrc/sigma.hip)
across library builds (tools/build_var.sh NAME DEFS sigma.hip): config-2
shapes (262,144 samples, 256 per ray), the same packed weights and
encodings; each library's avr_sigma_fwd is swapped in for the product's,
HIP events, interleaved rounds, and whether the outputs equal the first
library's bit for bit.

    python tools/xbench_sigma.py base=tools/_lib/libvar_sbase.so,x=tools/_lib/libvar_sx.so [--variant h1]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import _lib, sigma  # noqa: E402


class _Swap:
    """The product library with avr_sigma_fwd (and its error text) taken from `alt`."""

    def __init__(self, prod, alt):
        self.prod, self.alt = prod, alt
        fn = alt.avr_sigma_fwd
        fn.restype, fn.argtypes = _lib._SIGS["avr_sigma_fwd"]
        alt.avr_last_error.restype = ctypes.c_char_p

    def __getattr__(self, name):
        return getattr(self.alt if name in ("avr_sigma_fwd", "avr_last_error") else self.prod, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--variant", default="h1", choices=["h1", "meshrir", "raf"])
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--tile-cfg", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    dev = torch.device("cuda", 0)
    var = {"h1": sigma.MESHRIR_H1, "meshrir": sigma.MESHRIR, "raf": sigma.RAF}[a.variant]
    base_v = sigma.MESHRIR if var == sigma.MESHRIR_H1 else var
    N, S = 262144, 256
    g = torch.Generator(device=dev).manual_seed(1)
    ws = [torch.randn(M, K, device=dev, generator=g) * (2.0 / K) ** 0.5 for M, K, _, _ in sigma.SCHEDULE[var]]
    rnd = lambda rows, t: (torch.rand(rows, 40, device=dev, generator=g) * 2 - 1).to(t)  # noqa: E731
    if base_v == sigma.MESHRIR:
        inputs = [(rnd(N, torch.float16), 1)]
        extras = [(rnd(N // S, torch.float16), S), (rnd(1, torch.float16), N)]
    else:
        inputs = [(rnd(N, torch.float32), 1), (rnd(1, torch.float32), N)]
        extras = [(rnd(N // S, torch.float32), S), (rnd(1, torch.float32), N), (rnd(N, torch.float32), 1),
                  (rnd(1, torch.float32), N)]
    kw, out_w = {}, (128 if var == sigma.MESHRIR else 256)
    if var == sigma.MESHRIR_H1:
        extras, out_w = [], 512
        kw = dict(bias=torch.randn(N // S, 512, device=dev, generator=g) * 0.3, bias_div=S)
    packed = sigma.pack_layers(var, ws, dt)
    slope = 0.03 if var == sigma.RAF else 0.01
    prod = _lib.load()
    libs = []
    for item in a.libs.split(","):
        name, path = item.split("=", 1)
        libs.append((name, _Swap(prod, ctypes.CDLL(os.path.join(ROOT, path)))))

    def run():
        return sigma.sigma_fwd(var, packed, N, inputs, extras, out_w, slope, tile_cfg=a.tile_cfg, **kw)

    outs, times = {}, {n: [] for n, _ in libs}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    for name, lib in libs:
        _lib._lib = lib
        run()
        outs[name] = [t.clone() for t in run()]
    for _ in range(a.rounds):
        for name, lib in libs:
            _lib._lib = lib
            for e0, e1 in ev:
                e0.record()
                run()
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
    _lib._lib = prod
    ref = outs[libs[0][0]]
    for name, _ in libs:
        t = sorted(times[name])
        eq = all(torch.equal(x, y) for x, y in zip(outs[name], ref))
        print(json.dumps({"lib": name, "variant": a.variant, "dtype": a.dtype, "tile_cfg": a.tile_cfg,
                          "median_us": t[len(t) // 2], "min_us": t[0], "bitwise_equal_to_" + libs[0][0]: eq}),
              flush=True)


if __name__ == "__main__":
    main()
