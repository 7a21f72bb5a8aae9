"""Time the hash-grid backward (avr_hashgrid_bwd) on config-3 training
points: 4 RAF poses x 650 rays x 32 samples, the RAF position grid (20
levels, 2^18, base 16, fp16 encoding, fp16 upstream gradient), for each
points walked per lane group (AVR_HASHGRID_BWD_RUN, read at every launch),
interleaved over rounds; then per level at the default setting.

    python tools/probe_hashgrid_bwd.py [--iters 1,4,8,16,32] [--rounds 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import numpy as np
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
    ap.add_argument("--iters", default="1,4,8,16,32")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS["c3_raf_furnished_b4"]
    B = w.batch
    g = torch.Generator(device=dev).manual_seed(0)
    r = AVRRender(_Null(), **w.render)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    pts = r.sample(ro, tx)[0]
    x = ((pts.reshape(-1, 3) + 1) / 2).contiguous()
    N = x.size(0)
    enc = HashGridEncoding(3, RAF_MODEL["pos_encoding_sigma"], dtype=torch.float16).to(dev)
    L = enc.n_levels
    gout = (torch.randn(N, 2 * L, device=dev, generator=g) * 1e-2).half()
    gp = torch.zeros(enc.n_params, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def bwd(n_levels=L, off=enc._off, scale=enc._scale, res=enc._res, go=gout):
        _lib.call("avr_hashgrid_bwd", N, n_levels, x.data_ptr(), go.data_ptr(), _code(go.dtype),
                  off.ctypes.data, scale.ctypes.data, res.ctypes.data, gp.data_ptr(), st)

    nb = ctypes.c_int64()
    _lib.call("avr_hashgrid_bwd_workspace", N, L, enc._off.ctypes.data, ctypes.byref(nb))
    ws = torch.empty(nb.value, dtype=torch.uint8, device=dev)

    def bwd_part():
        _lib.call("avr_hashgrid_bwd_partitioned", N, L, x.data_ptr(), gout.data_ptr(), _code(gout.dtype),
                  enc._off.ctypes.data, enc._scale.ctypes.data, enc._res.ctypes.data, gp.data_ptr(),
                  ws.data_ptr(), nb.value, st)

    def time_us(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.reps

    iters = [int(v) for v in args.iters.split(",")]
    times = {str(it): [] for it in iters}
    times["partitioned"] = []
    for _ in range(args.rounds):
        for it in iters:
            os.environ["AVR_HASHGRID_BWD_RUN"] = str(it)
            times[str(it)].append(time_us(bwd))
        times["partitioned"].append(time_us(bwd_part))
        for dbg in (1, 2, 3):  # reduce pass without LDS adds / without the flush / neither
            os.environ["AVR_HG_BWD_DBG"] = str(dbg)
            times.setdefault(f"partitioned_dbg{dbg}", []).append(time_us(bwd_part))
        os.environ.pop("AVR_HG_BWD_DBG", None)
    # the gradients of the variants agree (summation order aside)
    outs = {}
    for it in iters:
        os.environ["AVR_HASHGRID_BWD_RUN"] = str(it)
        gp.zero_()
        bwd()
        torch.cuda.synchronize()
        outs[str(it)] = gp.clone()
    gp.zero_()
    bwd_part()
    torch.cuda.synchronize()
    outs["partitioned"] = gp.clone()
    # float64 scatter-add reference of the same gradient
    ref = outs[str(iters[0])]
    scale_ = float(ref.abs().max())
    # diagnostics of the reduce pass: the slowest slice and the butterfly count
    nbytes = nb.value
    ws[nbytes - 256:].zero_()
    os.environ["AVR_HG_BWD_DBG"] = "4"
    bwd_part()
    torch.cuda.synchronize()
    os.environ.pop("AVR_HG_BWD_DBG", None)
    d = ws[nbytes - 256:nbytes - 232].view(torch.int64).cpu().tolist()
    slowest_b, slowest_cycles = d[0] & ((1 << 24) - 1), d[0] >> 24
    # workspace offsets as bwd_layout lays them out (256-byte aligned segments)
    al = lambda v: (v + 255) // 256 * 256
    tp = int(sum(-(-int(sz) // 1024) for sz in np.diff(enc._off)))
    nch = -(-N // 512)
    o_tot = al(tp * nch * 4)
    o_ps = o_tot + al(tp * 4)
    o_sb = o_ps + al((tp + 1) * 4)
    totals = ws[o_tot:o_tot + 4 * tp].view(torch.int32).cpu().numpy()
    sb = ws[o_sb:o_sb + 4 * (tp + 1)].view(torch.int32).cpu().numpy()
    p_slow = int(np.searchsorted(sb, slowest_b, side="right") - 1)
    pbase = np.concatenate([[0], np.cumsum([-(-int(sz) // 1024) for sz in np.diff(enc._off)])])
    diag = {"slowest_cycles": slowest_cycles, "slowest_slice": slowest_b, "slowest_part": p_slow,
            "slowest_level": int(np.searchsorted(pbase, p_slow, side="right") - 1),
            "slowest_part_total": int(totals[p_slow]), "slowest_part_slices": int(sb[p_slow + 1] - sb[p_slow]),
            "butterfly_iters": d[1], "contribs": d[2], "total_slices": int(sb[-1]),
            "max_part_total": int(totals.max()), "mean_part_total": float(totals.mean())}
    # the slowest partition's keys, in the order the reduce wave reads them
    o_c = o_sb + al((tp + 1) * 4)  # (key, v0, v1) records
    ps = ws[o_ps:o_ps + 4 * (tp + 1)].view(torch.int32).cpu().numpy()
    k = ws[o_c + 12 * int(ps[p_slow]):o_c + 12 * int(ps[p_slow] + totals[p_slow])].view(torch.int32).view(-1, 3)[:, 0]
    k = k.cpu().numpy()
    rep, mx, dist = [], [], []
    for j in range(0, len(k), 64):
        u_, c_ = np.unique(k[j:j + 64], return_counts=True)
        rep.append(int((c_ > 1).sum()))
        mx.append(int(c_.max()))
        dist.append(len(u_))
    diag.update({"slow_repeated_keys_per_load_mean": float(np.mean(rep)), "slow_repeated_keys_per_load_max": int(max(rep)),
                 "slow_max_mult_mean": float(np.mean(mx)), "slow_distinct_per_load_mean": float(np.mean(dist)),
                 "slow_key_min": int(k.min()), "slow_key_max": int(k.max())})
    res = {"n_points": N, "levels": L, "rounds": args.rounds, "workspace_MB": nb.value / 2**20, "diag": diag,
           "us": {k: statistics.median(v) for k, v in times.items()},
           "max_abs_diff_vs_first": {k: float((v - ref).abs().max()) / scale_ for k, v in outs.items()}}
    os.environ.pop("AVR_HASHGRID_BWD_RUN", None)
    per = []
    for l in range(L):
        off = np.ascontiguousarray(enc._off[l:l + 2])
        sc = np.ascontiguousarray(enc._scale[l:l + 1])
        rs = np.ascontiguousarray(enc._res[l:l + 1])
        go = gout[:, 2 * l:2 * l + 2].contiguous()
        per.append(round(time_us(lambda: bwd(1, off, sc, rs, go)), 2))
    res["per_level_us"] = per
    res["per_level_sum_us"] = round(sum(per), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
