"""One width-512 ReLU layer: the hand-written GEMM (csrc/linear512.hip)
against hipBLASLt as the model runs it (with the shipped TunableOp solution
where the shape is listed), HIP events, interleaved rounds.

    python tools/bench_linear512.py [--rows 262144,2097152] [--dtype fp16] [--lib tools/_lib/libvar_x.so]
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

from avr_amd import _lib, model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="262144,2097152")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--libs", default="", help="name=path,... variant libraries timed beside the product's")
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    code = _lib.DTYPE_F16 if dt == torch.float16 else _lib.DTYPE_BF16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    w = torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    wf = torch.empty(512, 512, dtype=dt, device=dev)
    _lib.call("avr_linear512_pack_w", ctypes.c_void_p(w.to(dt).contiguous().data_ptr()), code,
              ctypes.c_void_p(wf.data_ptr()), st)
    libs = [("linear512", _lib.load().avr_linear512_relu_fwd)]
    for item in filter(None, a.libs.split(",")):
        name, path = item.split("=", 1)
        fn = ctypes.CDLL(os.path.join(ROOT, path)).avr_linear512_relu_fwd
        fn.restype, fn.argtypes = _lib._SIGS["avr_linear512_relu_fwd"]
        libs.append((name, fn))
    for M in (int(v) for v in a.rows.split(",")):
        x = torch.relu(torch.randn(M, 512, device=dev, generator=g)).to(dt)
        y = torch.empty_like(x)
        fns = {n: (lambda f=f: f(M, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wf.data_ptr()), code,
                                 ctypes.c_void_p(y.data_ptr()), st)) for n, f in libs}
        fns["hipblaslt"] = lambda: model._LinearReLU.apply(x, w, dt, True)
        with torch.no_grad():
            ref = model._LinearReLU.apply(x, w, dt, True).float()
            fns["linear512"]()
            torch.cuda.synchronize()
            diff = float(((y.float() - ref).abs() / torch.maximum(ref.abs(), ref.pow(2).mean().sqrt())).max())
            times = {n: [] for n in fns}
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.iters)]
            for _ in range(a.rounds):
                for n, fn in fns.items():
                    for e0, e1 in ev:
                        e0.record()
                        fn()
                        e1.record()
                    torch.cuda.synchronize()
                    times[n] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
        res = {"rows": M, "dtype": a.dtype, "max_rel_diff_vs_hipblaslt": diff}
        with torch.no_grad():  # variants against the product kernel, bit for bit
            fns["linear512"]()
            torch.cuda.synchronize()
            y0 = y.clone()
            for n, _ in libs[1:]:
                y.fill_(float("nan"))
                fns[n]()
                torch.cuda.synchronize()
                res[n + "_bitwise_equal"] = bool(torch.equal(y, y0))
        for n, v in times.items():
            v.sort()
            res[n + "_median_us"] = v[len(v) // 2]
            res[n + "_min_us"] = v[0]
        res["linear512_pflops"] = 2 * M * 512 * 512 / (res["linear512_median_us"] * 1e-6) / 1e15
        res["linear512_hbm_tbs"] = 2 * M * 512 * x.element_size() / (res["linear512_median_us"] * 1e-6) / 1e12
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
