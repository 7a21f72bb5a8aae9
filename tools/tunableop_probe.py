"""PyTorch TunableOp over the width-512 hidden layers (config 2, M = 262,144
rows): time torch._addmm_activation (hipBLASLt's default solution) against
the solution TunableOp picks after benchmarking every hipBLASLt / rocBLAS
candidate for the shape.  Writes the tuning to the given CSV.

    python tools/tunableop_probe.py OUT.csv [--dtype fp16]
"""
import json
import os
import sys

import torch


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    out = sys.argv[1]
    dt = torch.bfloat16 if "--dtype" in sys.argv and sys.argv[sys.argv.index("--dtype") + 1] == "bf16" else torch.float16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = 262144, 512, 512
    x = torch.relu(torch.randn(M, K, device=dev, generator=g)).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(dt)
    bias = torch.zeros(N, dtype=dt, device=dev)
    f_act = lambda: torch._addmm_activation(bias, x, w.t(), use_gelu=False)
    f_mm = lambda: torch.relu_(x @ w.t())
    base = {"addmm_activation": timeit(f_act), "mm+relu": timeit(f_mm)}
    ref = f_act().float()
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(out)
    torch.cuda.tunable.set_max_tuning_duration(2000)
    f_act()
    f_mm()
    torch.cuda.tunable.tuning_enable(False)
    tuned = {"addmm_activation": timeit(f_act), "mm+relu": timeit(f_mm)}
    same = bool(torch.equal(f_act().float(), ref))
    print(json.dumps({"dtype": str(dt), "default_us": base, "tunableop_us": tuned, "bitwise_equal": same}), flush=True)


if __name__ == "__main__":
    main()
