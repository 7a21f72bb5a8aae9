"""A/B timing of the partitioned hash-grid backward
(`avr_hashgrid_bwd_partitioned_set`) across library builds on config-3
training points (ray-ordered samples of 4 RAF poses, the RAF position grid,
fp32 encoding and upstream gradient as the training step runs it),
interleaved in one process; outputs compared with the first library's.

    python tools/xbench_hgbwd.py r5=tools/_lib/libab_hg_r5.so,cur=avr_amd/libavr_hip.so
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

from avr_amd import AVRRender, _lib  # noqa: E402
from avr_amd.encoding import HashGridEncoding, _code  # noqa: E402
from avr_amd.workloads import RAF_MODEL, WORKLOADS  # noqa: E402


class _Null(torch.nn.Module):
    def forward(self, *a, **k):
        raise RuntimeError


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[a.workload]
    g = torch.Generator(device=dev).manual_seed(0)
    r = AVRRender(_Null(), **w.render)
    ro = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    x = ((r.sample(ro, tx)[0].reshape(-1, 3) + 1) / 2).contiguous()
    N = x.size(0)
    enc = HashGridEncoding(3, RAF_MODEL["pos_encoding_sigma"], dtype=torch.float32).to(dev)
    L = enc.n_levels
    gout = torch.randn(N, 2 * L, device=dev, generator=g) * 1e-2
    st = torch.cuda.current_stream(dev).cuda_stream
    libs = []
    for item in a.libs.split(","):
        name, path = item.split("=", 1)
        lib = ctypes.CDLL(os.path.join(ROOT, path) if not os.path.isabs(path) else path)
        for fn in ("avr_hashgrid_bwd_partitioned_set", "avr_hashgrid_bwd_workspace"):
            getattr(lib, fn).restype, getattr(lib, fn).argtypes = _lib._SIGS[fn]
        lib.avr_last_error.restype = ctypes.c_char_p
        nb = ctypes.c_int64()
        assert lib.avr_hashgrid_bwd_workspace(N, L, enc._off.ctypes.data, ctypes.byref(nb)) == 0
        ws = torch.empty(max(1, nb.value), dtype=torch.uint8, device=dev)
        libs.append((name, lib, ws))
    outs, times = {}, {n: [] for n, _, _ in libs}

    def call(lib, ws, gp):
        rc = lib.avr_hashgrid_bwd_partitioned_set(N, L, x.data_ptr(), gout.data_ptr(), _code(gout.dtype),
                                                  enc._off.ctypes.data, enc._scale.ctypes.data,
                                                  enc._res.ctypes.data, gp.data_ptr(), ws.data_ptr(),
                                                  ws.numel(), st)
        if rc:
            raise RuntimeError(lib.avr_last_error().decode())

    for name, lib, ws in libs:
        gp = torch.full((enc.n_params,), float("nan"), device=dev)
        call(lib, ws, gp)
        call(lib, ws, gp)
        torch.cuda.synchronize()
        outs[name] = gp
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    gp = torch.empty(enc.n_params, device=dev)
    for _ in range(a.rounds):
        for name, lib, ws in libs:
            for e0, e1 in ev:
                e0.record()
                call(lib, ws, gp)
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
    ref = outs[libs[0][0]]
    scale = float(ref.abs().max())
    for name, _, _ in libs:
        t = sorted(times[name])
        o = outs[name]
        print(json.dumps({"lib": name, "workload": a.workload, "points": N, "levels": L, "median_us": t[len(t) // 2],
                          "min_us": t[0], "finite": bool(torch.isfinite(o).all()),
                          "max_abs_diff_rel_scale": float((o - ref).abs().max()) / scale}), flush=True)


if __name__ == "__main__":
    main()
