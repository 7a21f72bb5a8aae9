"""Interleaved A/B of two exact-head builds on the same inputs and box:
the current library against a previous one (csrc/build/libavr_exact_old.so,
built from an earlier commit's head_exact.hip by tools/build_ab_old.sh, with
that commit's ABI: no delay / queue arguments).  Config 2, fp16, the inputs
of one render_from_hidden call, captured inside the call.  One JSON line per
round and a summary.

    python tools/ab_exact.py [--rounds 5] [--iters 20]
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, _lib  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402

OLD = ctypes.CDLL(os.path.join(ROOT, "avr_amd", "csrc", "build", "libavr_exact_old.so"))
_vp, _i32 = ctypes.c_void_p, ctypes.c_int32
OLD.avr_head_fwd_exact.restype = ctypes.c_int
OLD.avr_head_fwd_exact.argtypes = [_vp, _i32, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp]


def arg(k, argv, d):
    return type(d)(argv[argv.index(k) + 1]) if k in argv else d


def main():
    rounds, iters = arg("--rounds", sys.argv, 5), arg("--iters", sys.argv, 20)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(19)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, 512
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(torch.float16)
    W = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
    r = AVRRender(None, **w.render)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    real = _lib.call
    res = {"new": [], "old": []}

    def call(name, *a):
        if name != "avr_head_fwd_exact":
            return real(name, *a)
        p, Bc, Kc, hp, Wf, code, perm, ws, cnt, delay, n_split, zpart, queue, st = a
        zp_old = torch.empty(n_split, Bc, S, T, dtype=torch.float32, device=dev)

        def new():
            real(name, *a)

        def old():
            rc = OLD.avr_head_fwd_exact(p, Bc, Kc, hp, Wf, code, perm, ws, cnt, n_split, zp_old.data_ptr(), st)
            assert rc == 0

        for f in (new, old, new, old):
            f()
        torch.cuda.synchronize()
        for k in range(rounds):
            for tag, f in (("new", new), ("old", old)) if k % 2 == 0 else (("old", old), ("new", new)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / iters
                res[tag].append(us)
                print(json.dumps({"round": k, "build": tag, "us": us}), flush=True)
        new()  # leave the new build's slabs for the render to finish with
        return None

    import avr_amd.renderer as rr
    rr._lib.call = call
    _lib.call = call
    with torch.no_grad():
        r.render_from_hidden(attn, h, W, torch.float16, geom)
    torch.cuda.synchronize()
    s = {k: sorted(v) for k, v in res.items()}
    print(json.dumps({"summary": "median us", "new": s["new"][len(s["new"]) // 2],
                      "old": s["old"][len(s["old"]) // 2], "new_min": s["new"][0], "old_min": s["old"][0]}),
          flush=True)


if __name__ == "__main__":
    main()
