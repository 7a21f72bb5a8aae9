"""Host-side cost of one eager config-2 render_ir (stub network): cProfile of
N unsynchronised renders, plus the wall time per render with and without a
synchronize after each (serial latency vs issue rate).

    python tools/host_probe.py [--n 400]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402
from bench import StubNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=dev).manual_seed(0)
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=dev, generator=g) * 0.1
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    r = AVRRender(StubNet(attn, sig), **w.render)
    with torch.no_grad():
        for _ in range(20):
            r.render_ir(ro, tx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.n):
            r.render_ir(ro, tx)
        t_issue = (time.perf_counter() - t0) / args.n
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / args.n
        t0 = time.perf_counter()
        for _ in range(args.n // 4):
            r.render_ir(ro, tx)
            torch.cuda.synchronize()
        t_serial = (time.perf_counter() - t0) / (args.n // 4)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.n):
            r.render_ir(ro, tx)
        pr.disable()
        torch.cuda.synchronize()
    print(f"issue {t_issue * 1e6:.1f} us/render, throughput {t_all * 1e6:.1f} us/render, "
          f"serial {t_serial * 1e6:.1f} us/render")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
