"""GPU probe: weight-gradient GEMM formulations for the MLP backward
(dW = gy^T x, gy [N, out], x [N, in], N ~ 1e5): host issue time and device
time of each, to pick the split-K strategy in avr_amd/model.py.

    python tools/mm_probe.py [--n 83200] [--dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=83200)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--interleave", action="store_true",
                    help="alternate all shapes every iteration (as a training step does)")
    ap.add_argument("--blas", default="", help="hipblaslt | cublas (rocBLAS)")
    args = ap.parse_args()
    if args.blas:
        torch.backends.cuda.preferred_blas_library(args.blas)
    if args.interleave:
        return interleaved(args)
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dev = torch.device("cuda", 0)
    rows = 4096
    for (o, i) in ((512, 512), (1600, 512), (512, 336), (128, 128)):
        gy = torch.randn(args.n, o, device=dev, dtype=dt)
        x = torch.randn(args.n, i, device=dev, dtype=dt)
        k = args.n // rows
        m = k * rows
        a_t = gy[:m].view(k, rows, o).transpose(1, 2)
        b = x[:m].view(k, rows, i)

        cands = {
            "mm_full": lambda: gy.t() @ x,
            "bmm_tview": lambda: torch.bmm(a_t, b).sum(0, dtype=torch.float32),
            "bmm_contig": lambda: torch.bmm(a_t.contiguous(), b).sum(0, dtype=torch.float32),
            "bmm_xT": lambda: torch.bmm(b.transpose(1, 2), gy[:m].view(k, rows, o)).sum(0, dtype=torch.float32),
            "matmul3d": lambda: torch.matmul(a_t, b).sum(0, dtype=torch.float32),
            "mm_loop": lambda: sum((gy[j * rows:(j + 1) * rows].t() @ x[j * rows:(j + 1) * rows]).float()
                                   for j in range(k)),
        }
        try:
            cands["bmm_f32out"] = lambda: torch.bmm(a_t, b, out_dtype=torch.float32).sum(0)
        except Exception:  # noqa: BLE001
            pass
        for name, fn in cands.items():
            try:
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                host = (time.perf_counter() - t0) / args.iters * 1e6
                e1.synchronize()
                dev_us = e0.elapsed_time(e1) / args.iters * 1e3
                print(json.dumps({"shape": [args.n, o, i], "case": name, "host_us": round(host, 1),
                                  "dev_us": round(dev_us, 1)}), flush=True)
            except Exception as exc:  # noqa: BLE001
                print(json.dumps({"shape": [args.n, o, i], "case": name, "error": str(exc)[:200]}))


def interleaved(args):
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dev = torch.device("cuda", 0)
    rows = 4096
    shapes = ((512, 512), (1600, 512), (512, 336), (128, 128), (256, 128), (128, 80), (512, 512),
              (1, 256), (256, 128), (128, 120))
    data = [(torch.randn(args.n, o, device=dev, dtype=dt), torch.randn(args.n, i, device=dev, dtype=dt))
            for o, i in shapes]
    k = args.n // rows
    m = k * rows

    def bmm_all():
        for gy, x in data:
            torch.bmm(gy[:m].view(k, rows, -1).transpose(1, 2), x[:m].view(k, rows, -1))

    def mm_all():
        for gy, x in data:
            gy.t() @ x

    for name, fn in (("bmm", bmm_all), ("mm", mm_all)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        host = (time.perf_counter() - t0) / args.iters / len(shapes) * 1e6
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) / args.iters / len(shapes) * 1e6
        print(json.dumps({"interleaved": name, "blas": args.blas or "default",
                          "host_us_per_call": round(host, 1), "wall_us_per_call": round(tot, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
