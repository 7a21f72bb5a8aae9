"""A/B timing of the fused two-layer width-512 kernel (`avr_mlp512x2_fwd`,
csrc/mlp512.hip) across library builds (tools/build_var.sh with
EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1"), same packed weights and rows,
HIP events, interleaved rounds; per library the median / min and whether
the output equals the first library's bit for bit.

    python tools/xbench_mlp.py base=tools/_lib/libvar_mbase.so,dma=tools/_lib/libvar_mdma.so [--rows 262144]
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
    ap.add_argument("libs")
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    code = _lib.DTYPE_F16 if dt == torch.float16 else _lib.DTYPE_BF16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.relu(torch.randn(a.rows, 512, device=dev, generator=g)).to(dt)
    w1 = (torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5).to(dt)
    w2 = (torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5).to(dt)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    wf = torch.empty(2, 512, 512, dtype=dt, device=dev)
    _lib.call("avr_mlp512x2_pack_w", ctypes.c_void_p(w1.data_ptr()), ctypes.c_void_p(w2.data_ptr()), code,
              ctypes.c_void_p(wf.data_ptr()), st)
    y = torch.empty_like(x)
    libs = []
    for item in a.libs.split(","):
        name, path = item.split("=", 1)
        lib = ctypes.CDLL(os.path.join(ROOT, path))
        fn = lib.avr_mlp512x2_fwd
        fn.restype, fn.argtypes = _lib._SIGS["avr_mlp512x2_fwd"]
        libs.append((name, fn))
    args = (a.rows, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wf.data_ptr()), code,
            ctypes.c_void_p(y.data_ptr()), st)
    outs, times = {}, {n: [] for n, _ in libs}
    for name, fn in libs:
        y.fill_(float("nan"))
        assert fn(*args) == 0 and fn(*args) == 0
        torch.cuda.synchronize()
        outs[name] = y.clone()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    for _ in range(a.rounds):
        for name, fn in libs:
            for e0, e1 in ev:
                e0.record()
                fn(*args)
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
    ref = outs[libs[0][0]]
    for name, _ in libs:
        t = sorted(times[name])
        print(json.dumps({"lib": name, "rows": a.rows, "dtype": a.dtype, "median_us": t[len(t) // 2], "min_us": t[0],
                          "pflops": 4 * a.rows * 512 * 512 / (t[len(t) // 2] * 1e-6) / 1e15,
                          "bitwise_equal_to_" + libs[0][0]: bool(torch.equal(outs[name], ref))}), flush=True)


if __name__ == "__main__":
    main()
