"""Host-side profile of the bench's eager render (config 2, stub network):
cProfile over N render_ir calls issued without synchronising, top functions
by own time.  Shows where the ~0.075-0.09 ms of host issue per pose goes.

    python tools/host_profile.py [--n 300]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=dev).manual_seed(0)
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=dev, generator=g) * 0.1
    r = AVRRender(bench.StubNet(attn, sig), **w.render)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    with torch.no_grad():
        for _ in range(20):
            r.render_ir(ro, tx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.n):
            r.render_ir(ro, tx)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"host issue {1e3 * (t1 - t0) / args.n:.4f} ms per pose (no profiler)")
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.n):
            r.render_ir(ro, tx)
        pr.disable()
        torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
