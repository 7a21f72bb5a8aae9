"""A/B timing of the exact head kernel (`avr_head_fwd_exact`) across library
builds, on the same config-2 inputs, interleaved in one process.

The geometry (weights, delays, the delay sort, the packed W) comes from the
product library; each library under test is then called with exactly the
same arguments.  Per library: the median and min of HIP-event timings over
`--iters` back-to-back launches per round, `--rounds` rounds interleaved,
and whether its output equals the first library's bit for bit.

    python tools/xbench_exact.py r5=tools/_lib/libab_r5.so,hold=tools/_lib/libab_hold.so \
        [--workload c5_simu_4096x512x2048 --shard-of 8]

(tools/build_ab.sh builds the libraries: errors.cpp + head_exact.hip from a
git revision or the working tree.)
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
from avr_amd.renderer import _ptr, _stream, _weights, ctypes_ref, get_tables  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def setup(workload, dtype, K, seed=19, shard_of=1):
    from avr_amd.parallel import shard_range

    w = WORKLOADS[workload]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    r0, r1 = shard_range(R, 0, max(1, shard_of))
    R = r1 - r0
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(seed)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    attn = torch.rand(B, R * S, device=dev, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(dtype)
    W = (torch.randn(T, K, device=dev, generator=g) / K ** 0.5).to(dtype)
    r = AVRRender(None, **w.render)
    if shard_of > 1:
        r.ray_range = (r0, r1)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    p = r._params(T, R)
    tables = get_tables(p, dev)
    st = _stream(dev)
    pref = ctypes_ref(p)
    code = _lib.DTYPE_F16 if dtype == torch.float16 else _lib.DTYPE_BF16
    wts, delay = _weights(p, attn, geom["rays_o"], geom["position_tx"], geom["dirs"], tables, st)
    perm = torch.empty(B, S, R, dtype=torch.int32, device=dev)
    ws = torch.empty(B, S, R, dtype=torch.float32, device=dev)
    cnt = torch.empty(B, S, T, dtype=torch.int32, device=dev)
    _lib.call("avr_head_sort", pref, B, _ptr(wts), _ptr(delay), _ptr(perm), _ptr(ws), _ptr(cnt), st)
    ns, wbytes = ctypes.c_int32(0), ctypes.c_int64(0)
    _lib.call("avr_head_exact_layout", pref, B, K, code, ctypes.byref(ns), ctypes.byref(wbytes))
    Wf = torch.empty(wbytes.value // 2, dtype=dtype, device=dev)
    _lib.call("avr_head_pack_w_exact", pref, K, _ptr(W), code, _ptr(Wf), st)
    part = torch.empty(ns.value, B, S, T, dtype=torch.float32, device=dev)
    queue = torch.empty(256, dtype=torch.int32, device=dev)
    args = (pref, B, K, _ptr(h), _ptr(Wf), code, _ptr(perm), _ptr(ws), _ptr(cnt), _ptr(delay), ns.value,
            _ptr(part), _ptr(queue), st)
    keep = (h, Wf, perm, ws, cnt, delay, queue, wts, p)
    return args, part, keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", help="name=path,name=path,... (the first is the reference for equality)")
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shard-of", type=int, default=1, help="rank 0's ray shard of an N-rank split")
    a = ap.parse_args()
    dtype = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    libs = []
    for item in a.libs.split(","):
        name, path = item.split("=", 1)
        lib = ctypes.CDLL(os.path.join(ROOT, path) if not os.path.isabs(path) else path)
        fn = lib.avr_head_fwd_exact
        fn.restype, fn.argtypes = _lib._SIGS["avr_head_fwd_exact"]
        err = lib.avr_last_error
        err.restype = ctypes.c_char_p
        libs.append((name, fn, err))
    args, part, keep = setup(a.workload, dtype, a.K, shard_of=a.shard_of)
    outs, times = {}, {n: [] for n, _, _ in libs}

    def call(fn, err):
        rc = fn(*args)
        if rc != 0:
            raise RuntimeError(err().decode())

    for name, fn, err in libs:  # warm + outputs
        part.fill_(float("nan"))
        call(fn, err)
        call(fn, err)
        torch.cuda.synchronize()
        outs[name] = part.clone()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    for _ in range(a.rounds):
        for name, fn, err in libs:
            for e0, e1 in ev:
                e0.record()
                call(fn, err)
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
    ref = outs[libs[0][0]]
    for name, _, _ in libs:
        t = sorted(times[name])
        print(json.dumps({"lib": name, "workload": a.workload, "dtype": a.dtype, "median_us": t[len(t) // 2],
                          "min_us": t[0], "n": len(t), "bitwise_equal_to_" + libs[0][0]: bool(torch.equal(outs[name], ref)),
                          "finite": bool(torch.isfinite(outs[name]).all()),
                          "max_abs_diff": float((outs[name] - ref).abs().max()),
                          "rel_l2_diff": float((outs[name] - ref).norm() / ref.norm())}), flush=True)


if __name__ == "__main__":
    main()
