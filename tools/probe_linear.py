"""GPU probe: the width-512 hidden layer at config 2 (M = 262,144 rows),
avr_linear_relu_fwd against hipBLASLt's torch._addmm_activation (the form
model.py uses), HIP-event timing and agreement.

    python tools/probe_linear.py [--dtype fp16] [--iters 20]
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

# the shape switch (AVR_LINEAR_SHAPE_PROBE) is read only by the shape-probe
# build (`make -C avr_amd/csrc shapes`, no phase clocks); the shipped library
# always runs shape 0
PROBE = ctypes.CDLL(os.path.join(ROOT, "tools", "_lib", "libavr_shapes.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--M", type=int, default=262144)
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="0,1,2", help="AVR_LINEAR_SHAPE_PROBE values, interleaved --reps times")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=200)
    args = ap.parse_args()
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    code = _lib.DTYPE_F16 if dt == torch.float16 else _lib.DTYPE_BF16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = args.M, args.N, 512
    x = torch.relu(torch.randn(M, K, device=dev, generator=g)).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(dt)
    bias = torch.zeros(N, dtype=dt, device=dev)
    y = torch.empty(M, N, dtype=dt, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    wf = torch.empty_like(w)
    _lib.load()
    PROBE.avr_linear_relu_fwd.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p]
    PROBE.avr_linear_pack_w.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                        ctypes.c_void_p, ctypes.c_void_p]
    assert PROBE.avr_linear_pack_w(N, K, w.data_ptr(), code, wf.data_ptr(), st) == 0

    def ours():
        assert PROBE.avr_linear_relu_fwd(M, N, K, x.data_ptr(), wf.data_ptr(), code, 1, y.data_ptr(), st) == 0
        return y

    def blas():
        return torch._addmm_activation(bias, x, w.t(), use_gelu=False)

    for _ in range(args.warmup):  # clocks up before anything is timed
        ours()
        blas()
    torch.cuda.synchronize()
    runs = []
    for _ in range(args.reps):
        runs += [("avr_linear_relu_fwd", ours, d) for d in args.shapes.split(",")] + [("hipblaslt_addmm_activation", blas, "0")]
    for name, fn, dbg in runs:
        os.environ["AVR_LINEAR_SHAPE_PROBE"] = dbg
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        print(json.dumps({"kernel": name, "shape": int(dbg), "dtype": args.dtype, "M": M, "N": N, "K": K, "us": ms * 1e3,
                          "pflops": 2 * M * N * K / (ms * 1e-3) / 1e15}), flush=True)
    a, b = ours().float(), blas().float()
    print(json.dumps({"equal_fraction": float((a == b).float().mean()),
                      "max_rel": float(((a - b).abs() / b.abs().clamp_min(1e-3)).max())}), flush=True)


if __name__ == "__main__":
    main()
