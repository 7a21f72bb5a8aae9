"""GPU probe: the linear head's forward partials z[b,s,t] (summed over the
feature slices) from avr_head_fwd against a torch statement of the same sum
on the sorted rays, per t-tile of 32, for the band form (AVR_HEAD_BAND=1) and
the feature-block form (0).

    python tools/probe_band_z.py [--case raf|c2] [--dtype bf16]
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
from avr_amd import renderer as rd  # noqa: E402
from avr_amd.workloads import RAF, WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="raf")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--cols", type=int, default=8)
    ap.add_argument("--forms", default="1,0", help="0: feature blocks, 1: band, 1<d>: band with AVR_HEAD_BAND_DBG=d")
    args = ap.parse_args()
    dt = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    dev = torch.device("cuda", 0)
    if args.case == "raf":
        cfg, B, T, K = dict(RAF, n_azi=36, n_ele=18, n_samples=32), 1, 1600, 512
    else:
        w = WORKLOADS["c2_meshrir_1024x256x512"]
        cfg, B, T, K = dict(w.render), 1, w.T, 512
    r = AVRRender(None, exact_head=False, **cfg)
    R = cfg["n_azi"] * cfg["n_ele"] + 2
    S = cfg["n_samples"]
    g = torch.Generator(device=dev).manual_seed(3)
    ro = torch.rand(B, 3, device=dev, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=dev, generator=g) * 2 - 1
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    attn = (torch.rand(B, R * S, device=dev, generator=g) * 2).contiguous()
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(dt).contiguous()
    Wm = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
    W = Wm.to(dt).contiguous()
    p = r._params(T, R)
    tables = rd.get_tables(p, dev)
    st = rd._stream(dev)
    pref = rd.ctypes_ref(p)
    code = rd._dtype_code(h)
    w, delay = rd._weights(p, attn, geom["rays_o"], geom["position_tx"], geom["dirs"], tables, st)
    perm = torch.empty(B, S, R, dtype=torch.int32, device=dev)
    ws = torch.empty(B, S, R, dtype=torch.float32, device=dev)
    cnt = torch.empty(B, S, T, dtype=torch.int32, device=dev)
    _lib.call("avr_head_sort", pref, B, rd._ptr(w), rd._ptr(delay), rd._ptr(perm), rd._ptr(ws), rd._ptr(cnt), st)
    Wp = torch.empty_like(W)
    _lib.call("avr_head_pack_w", pref, B, K, rd._ptr(W), code, rd._ptr(Wp), st)
    torch.cuda.synchronize()
    hs = h.view(B, R, S, K)
    cols = torch.linspace(0, S - 1, args.cols).long().tolist()
    refs = {}
    for s in cols:
        n = int(cnt[0, s, T - 1])
        rays = perm[0, s, :n].long()
        x = hs[0, rays, s, :].double() @ W.double().t()  # [n, T]
        wz = ws[0, s, :n].double()[:, None] * x
        cz = torch.cat([torch.zeros(1, T, dtype=torch.float64, device=dev), wz.cumsum(0)], 0)
        c = cnt[0, s].long()
        refs[s] = cz.gather(0, c[None, :])[0]  # z[t] = sum_{p < cnt[t]}
    for form in args.forms.split(","):
        os.environ["AVR_HEAD_BAND"] = "0" if form == "0" else "1"
        os.environ["AVR_HEAD_BAND_DBG"] = "0" if form in ("0", "1") else form[1:]
        ns = ctypes.c_int32(0)
        _lib.call("avr_head_splits", pref, B, K, code, ctypes.byref(ns))
        part = torch.full((ns.value, B, S, T), float("nan"), device=dev)
        _lib.call("avr_head_fwd", pref, B, K, rd._ptr(h), rd._ptr(Wp), code, rd._ptr(perm), rd._ptr(ws),
                  rd._ptr(cnt), ns.value, rd._ptr(part), st)
        torch.cuda.synchronize()
        z = part.double().sum(0)
        for s in cols:
            lim = int(T - 1 - tables.shift[s]) if hasattr(tables, "shift") else T
            ref = refs[s].clone()
            ref[lim:] = 0
            d = (z[0, s] - ref).abs()
            tiles = [float(d[i:i + 32].max() / ref.abs().max().clamp_min(1e-30)) for i in range(0, T, 32)]
            bad = [i for i, e in enumerate(tiles) if e > 1e-5]
            print(json.dumps({"band": form, "s": s, "n_live": int(cnt[0, s, T - 1]), "lim": lim,
                              "rel_l2": float((z[0, s] - ref).norm() / ref.norm().clamp_min(1e-30)),
                              "bad_tiles": bad[:12], "n_bad": len(bad),
                              "nan": bool(torch.isnan(z[0, s]).any())}), flush=True)
    os.environ.pop("AVR_HEAD_BAND", None)


if __name__ == "__main__":
    main()
