"""GPU probe: time the fused-head kernels in isolation at a workload's shape,
with phases switched off through AVR_HEAD_DBG (bit 0 scatter, 1 scan,
2 contraction) to see where the time goes.

    python tools/probe_head.py [--workload c3_raf_furnished_b4] [--K 512]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dbg", default="0,1,2,4,3,5,6,7")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, args.K
    r = AVRRender(None, **w.render)
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    _, _, _, _, geom = r.sample(ro, tx)
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(torch.bfloat16)
    W = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
    for dbg in args.dbg.split(","):
        os.environ["AVR_HEAD_DBG"] = dbg
        for _ in range(2):
            r.render_from_hidden(attn, h, W, torch.bfloat16, geom)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            r.render_from_hidden(attn, h, W, torch.bfloat16, geom)
        e1.record()
        e1.synchronize()
        print(json.dumps({"workload": w.name, "dbg": int(dbg),
                          "render_ms": e0.elapsed_time(e1) / args.iters}), flush=True)
    os.environ.pop("AVR_HEAD_DBG", None)


if __name__ == "__main__":
    main()
