"""GPU sweep of the MLP weight-gradient kernel's workgroup target
(AVR_WGRAD_WGS, read at every call) on the training shapes.

    python tools/tune_wgrad.py [--n 83200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd.model import _wgrad_hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=83200)
    ap.add_argument("--targets", default="512,1024,2048")
    ap.add_argument("--xcd", default="0,1")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    shapes = ((512, 512), (1600, 512), (512, 336), (256, 128), (128, 128), (128, 80))
    data = [(torch.randn(args.n, m, device=dev).to(torch.bfloat16),
             torch.randn(args.n, k, device=dev).to(torch.bfloat16)) for m, k in shapes]
    for tgt, xcd in [(t, x) for t in args.targets.split(",") for x in args.xcd.split(",")]:
        os.environ["AVR_WGRAD_WGS"] = tgt
        os.environ["AVR_WGRAD_XCD"] = xcd
        for (m, k), (gy, x) in zip(shapes, data):
            _wgrad_hip(gy, x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                _wgrad_hip(gy, x)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / args.iters * 1e3
            print(json.dumps({"target": int(tgt), "xcd": int(xcd), "N": args.n, "M": m, "K": k, "us": round(us, 1),
                              "TFLOPs": round(2 * args.n * m * k / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
