"""Time the fused signal head at config 2 (1024 rays x 256 samples, T=1022,
K=512): the exact (rounding) MFMA head against the linear head, 16-bit h.
Run under rocprofv3 --kernel-trace --stats for per-kernel times."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--modes", default="exact,linear")
    args = ap.parse_args()
    dtype = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    w = WORKLOADS[args.workload]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, args.K
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(19)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(dtype)
    W = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
    for mode in args.modes.split(","):
        r = AVRRender(None, exact_head=(mode == "exact"), **w.render)
        torch.manual_seed(5)
        _, _, _, _, geom = r.sample(ro, tx)
        with torch.no_grad():
            for _ in range(3):
                r.render_from_hidden(attn, h, W, dtype, geom)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                r.render_from_hidden(attn, h, W, dtype, geom)
            torch.cuda.synchronize()
        print(f"{mode}: {(time.perf_counter() - t0) * 1e3 / args.iters:.3f} ms per render", flush=True)


if __name__ == "__main__":
    main()
