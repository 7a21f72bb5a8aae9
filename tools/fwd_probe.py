"""GPU probe: forward MLP layer y = relu(x W^T) at the config-2 inference
shape (N = 262144 rows, 512 wide, bf16), as the network runs it today and
with the activation in the GEMM epilogue.

    python tools/fwd_probe.py [--n 262144] [--k 512] [--m 512]
"""
from __future__ import annotations

import argparse
import json

import torch


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    x = torch.randn(args.n, args.k, device=dev, dtype=dt)
    w = torch.randn(args.m, args.k, device=dev, dtype=dt) / args.k ** 0.5
    zb = torch.zeros(args.m, device=dev, dtype=dt)
    flops = 2 * args.n * args.k * args.m
    res = {"n": args.n, "k": args.k, "m": args.m}
    res["gemm_us"] = bench(lambda: x @ w.t(), args.iters)
    res["gemm_relu_us"] = bench(lambda: torch.relu(x @ w.t()), args.iters)
    res["gemm_relu_inplace_us"] = bench(lambda: torch.relu_(x @ w.t()), args.iters)
    try:
        y = torch._addmm_activation(zb, x, w.t(), use_gelu=False)
        ok = torch.equal(y, torch.relu(x @ w.t() + zb))
        res["addmm_act_us"] = bench(lambda: torch._addmm_activation(zb, x, w.t(), use_gelu=False),
                                    args.iters)
        res["addmm_act_exact"] = bool(ok)
    except Exception as e:  # noqa: BLE001
        res["addmm_act_error"] = str(e)[:200]
    res["linear_us"] = bench(lambda: torch.nn.functional.linear(x, w), args.iters)
    for k in list(res):
        if k.endswith("_us"):
            res[k.replace("_us", "_tflops")] = flops / (res[k] * 1e-6) / 1e12
    print(json.dumps(res))


if __name__ == "__main__":
    main()
