"""avr_linear_wgrad of the product library against variant builds
(tools/build_var.sh ... mlp.hip), same inputs, HIP events, interleaved.

    python tools/xbench_wgrad.py --libs name=path,... [--shape 83200,512,512]
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

from avr_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="83200,512,512")
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N, M, K = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    gy = torch.randn(N, M, device=dev, generator=g).bfloat16()
    x = torch.randn(N, K, device=dev, generator=g).bfloat16()
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    libs = [("product", _lib.load())]
    for item in filter(None, a.libs.split(",")):
        name, path = item.split("=")
        libs.append((name, ctypes.CDLL(os.path.join(ROOT, path))))
    outs, times = {}, {n: [] for n, _ in libs}
    splits = {}
    for name, lib in libs:
        sp = ctypes.c_int32(0)  # each library's own split count and workspace
        assert lib.avr_linear_wgrad_splits(ctypes.c_int64(N), M, K, ctypes.byref(sp)) == 0
        splits[name] = sp.value
        ws = torch.empty(sp.value * M * K, dtype=torch.float32, device=dev)
        out = torch.empty(M, K, dtype=torch.float32, device=dev)
        f = lib.avr_linear_wgrad
        f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 3 + [ctypes.c_int32] + \
            [ctypes.c_void_p] * 2
        call = (lambda f=f, out=out, ws=ws, n=sp.value: f(N, M, K, gy.data_ptr(), x.data_ptr(), ws.data_ptr(), n,
                                                          out.data_ptr(), st))
        outs[name] = (call, out, ws)
    for _ in range(a.rounds):
        for name, (call, out, _) in outs.items():
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                assert call() == 0
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / a.iters)
    ref = outs["product"][1]
    for name in times:
        t = sorted(times[name])
        same = torch.equal(outs[name][1], ref)
        close = float((outs[name][1] - ref).norm() / ref.norm())
        print(json.dumps(dict(variant=name, shape=[N, M, K], splits=splits[name], us_median=t[len(t) // 2], us_all=t,
                              GBps=(N * M + N * K) * 2 / t[len(t) // 2] / 1e3,
                              bitwise_equal=bool(same), rel_diff=close)))


if __name__ == "__main__":
    main()
