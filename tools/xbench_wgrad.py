"""A/B timing of the split-K weight gradient (`avr_linear_wgrad`, kernel +
finalize) across library builds at the training step's shapes, interleaved
in one process (HIP events); outputs compared bitwise with the first
library's.

    python tools/xbench_wgrad.py old=tools/_lib/libab_wg_old.so,cur=avr_amd/libavr_hip.so
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

SHAPES = [(83200, 512, 512), (83200, 512, 416), (147712, 512, 512), (83200, 256, 128), (83200, 128, 128),
          (83200, 128, 80)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    libs = []
    for item in a.libs.split(","):
        name, path = item.split("=", 1)
        lib = ctypes.CDLL(path if os.path.isabs(path) else os.path.join(ROOT, path))
        for fn in ("avr_linear_wgrad", "avr_linear_wgrad_splits"):
            getattr(lib, fn).restype, getattr(lib, fn).argtypes = _lib._SIGS[fn]
        lib.avr_last_error.restype = ctypes.c_char_p
        libs.append((name, lib))
    for N, M, K in SHAPES:
        g = torch.Generator(device=dev).manual_seed(N + M + K)
        gy = torch.randn(N, M, device=dev, generator=g).to(torch.bfloat16)
        x = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
        runs = []
        for name, lib in libs:
            sp = ctypes.c_int32(0)
            assert lib.avr_linear_wgrad_splits(N, M, K, ctypes.byref(sp)) == 0
            ws = torch.empty(sp.value * M * K, dtype=torch.float32, device=dev)
            out = torch.empty(M, K, dtype=torch.float32, device=dev)

            def call(lib=lib, ws=ws, out=out, n_sp=sp.value):
                rc = lib.avr_linear_wgrad(N, M, K, gy.data_ptr(), x.data_ptr(), ws.data_ptr(), n_sp,
                                          out.data_ptr(), st)
                if rc:
                    raise RuntimeError(lib.avr_last_error().decode())
            runs.append((name, call, out, sp.value))
        times = {n: [] for n, _, _, _ in runs}
        for _ in range(a.rounds):
            for name, call, _, _ in runs:
                call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        ref = runs[0][2]
        for name, _, out, n_sp in runs:
            print(json.dumps({"lib": name, "N": N, "M": M, "K": K, "splits": n_sp, "min_us": min(times[name]),
                              "bitwise_equal_to_first": bool(torch.equal(out, ref))}), flush=True)


if __name__ == "__main__":
    main()
