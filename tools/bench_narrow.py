"""avr_narrow_mm against what it replaces, at the training step's narrow
shapes: forward relu(x W^T) (hipBLASLt _addmm_activation, tuned where the
shipped file lists the shape) and data gradient g W (+ threshold_backward
for the masked form).  HIP events.

    python tools/bench_narrow.py [--rows 83200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import model as M  # noqa: E402


def t_us(fn, it=30):
    """GPU time per call: the calls are queued behind a spin kernel, so host
    issue time (ctypes, TunableOp window) does not show between them."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(2e7))
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=83200)
    ap.add_argument("--libs", default="", help="name=path,... variant libraries: their avr_narrow_mm timed too")
    a = ap.parse_args()
    import ctypes

    variants = []
    for item in filter(None, a.libs.split(",")):
        name, path = item.split("=")
        f = ctypes.CDLL(os.path.join(ROOT, path)).avr_narrow_mm
        f.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        variants.append((name, f))
    dev = torch.device("cuda", 0)
    N = a.rows
    g = torch.Generator(device=dev).manual_seed(0)
    for (inp, out) in [(80, 128), (128, 128), (128, 256), (256, 128)]:
        x = torch.relu(torch.randn(N, inp, device=dev, generator=g)).bfloat16()
        w = (torch.randn(out, inp, device=dev, generator=g) / inp ** 0.5).bfloat16()
        gy = torch.randn(N, out, device=dev, generator=g).bfloat16()
        bias = torch.zeros(out, dtype=torch.bfloat16, device=dev)

        def fwd_blas():
            if M._tuned_gemm(x, w):
                with M._tuned_window():
                    return torch._addmm_activation(bias, x, w.t(), use_gelu=False)
            return torch._addmm_activation(bias, x, w.t(), use_gelu=False)

        r = dict(rows=N, inp=inp, out=out,
                 fwd_narrow_us=t_us(lambda: M._narrow(x, w, 1)), fwd_blas_us=t_us(fwd_blas),
                 dgrad_narrow_us=t_us(lambda: M._narrow(gy, w.t(), 0)), dgrad_blas_us=t_us(lambda: M._mm_dgrad(gy, w)),
                 dgrad_mask_narrow_us=t_us(lambda: M._narrow(gy, w.t(), 2, x)),
                 dgrad_mask_blas_us=t_us(lambda: torch.ops.aten.threshold_backward(M._mm_dgrad(gy, w), x, 0)))
        r["fwd_bytes_GBps_narrow"] = N * (inp + out) * 2 / r["fwd_narrow_us"] / 1e3
        st = torch.cuda.current_stream(dev).cuda_stream
        wt = w.t().contiguous()
        for name, f in variants:
            yv = torch.empty(N, out, dtype=torch.bfloat16, device=dev)
            gv = torch.empty(N, inp, dtype=torch.bfloat16, device=dev)
            r[f"fwd_{name}_us"] = t_us(lambda: f(N, inp, out, x.data_ptr(), w.data_ptr(), 2, 1, None, yv.data_ptr(), st))
            r[f"dgrad_mask_{name}_us"] = t_us(lambda: f(N, out, inp, gy.data_ptr(), wt.data_ptr(), 2, 2, x.data_ptr(),
                                                        gv.data_ptr(), st))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
