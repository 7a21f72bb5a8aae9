"""GPU sweep of the backward ray reduction's launch shape (run on the box).

Times avr_ray_reduce_bwd directly through the C-ABI for several wave targets
(AVR_RB_WAVES, read at every launch), interleaved over rounds, next to a
plain device copy of the same tensor (the read+write stream ceiling).

    python tools/tune_bwd.py [--workload c3_raf_furnished_b4] [--waves 1024,2048,4096,8192]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import _lib  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    ap.add_argument("--waves", default="2048,8192,16384,65536")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="")
    ap.add_argument("--nts", default="0,1")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w_ = WORKLOADS[args.workload]
    if args.dtype:
        w_ = w_.replace(signal_dtype=args.dtype, attn_dtype=args.dtype)
    B, R, S, T = w_.batch, w_.n_rays, w_.n_samples, w_.T
    dt = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}[w_.signal_dtype]
    code = {torch.float32: _lib.DTYPE_F32, torch.float16: _lib.DTYPE_F16,
            torch.bfloat16: _lib.DTYPE_BF16}[dt]
    g = torch.Generator(device=dev).manual_seed(0)
    sig = (torch.randn(B, R * S, T, device=dev, generator=g) * 0.1).to(dt)
    gsig = torch.empty_like(sig)
    gz = torch.randn(B, S, T, device=dev, generator=g)
    w = torch.rand(B, R, S, device=dev, generator=g)
    delay = torch.randint(0, T // 2, (B, R, S), device=dev, dtype=torch.int32, generator=g)
    gw = torch.empty(B, R, S, device=dev)
    p = _lib.render_params(w_.render, T)
    import ctypes
    pref = ctypes.byref(p)
    st = torch.cuda.current_stream(dev).cuda_stream
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run_bwd():
        _lib.call("avr_ray_reduce_bwd", pref, B, ptr(sig), code, ptr(gz), ptr(w), ptr(delay),
                  ptr(gsig), ptr(gw), st)

    def run_copy():
        gsig.copy_(sig)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / args.iters * 1e3  # us

    nbytes = 2 * sig.numel() * sig.element_size()
    waves = [int(x) for x in args.waves.split(",")]
    res = {("copy",): []}
    ntss = [int(x) for x in args.nts.split(",")]
    res.update({(wv, n): [] for wv in waves for n in ntss})
    for _ in range(args.rounds):
        res[("copy",)].append(timed(run_copy))
        for wv in waves:
            for n in ntss:
                os.environ["AVR_RB_WAVES"] = str(wv)
                os.environ["AVR_RB_NTS"] = str(n)
                res[(wv, n)].append(timed(run_bwd))
    os.environ.pop("AVR_RB_WAVES", None)
    os.environ.pop("AVR_RB_NTS", None)
    for k, v in res.items():
        us = statistics.median(v)
        print(json.dumps({"workload": w_.name, "dtype": w_.signal_dtype, "case": "/".join(map(str, k)),
                          "us": round(us, 1), "TBps": round(nbytes / us / 1e6, 3)}))


if __name__ == "__main__":
    main()
