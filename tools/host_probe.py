"""Host-side cost of the training step's Python layer plumbing, per call
(GPU work queued behind a spin kernel, so only issue time is timed): the
TunableOp window, a ctypes entry, torch.empty, and one _LinearReLU layer's
forward + backward at config-3 rows with and without the tuned-GEMM window.

    python tools/host_probe.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import model as M  # noqa: E402
from avr_amd.options import KernelOptions  # noqa: E402


def per_call_us(fn, n=1000, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e9))  # keep the GPU busy: queued work does not block issue
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return dt


def main():
    dev = torch.device("cuda", 0)
    res = {}
    M._enable_tuned_gemms(dev)

    def win():
        with M._tuned_window():
            pass
    res["tuned_window_us"] = per_call_us(win)
    res["torch_empty_us"] = per_call_us(lambda: torch.empty(1024, device=dev))
    from avr_amd import _lib
    lib = _lib.load()
    res["ctypes_last_error_us"] = per_call_us(lambda: lib.avr_last_error())
    rows = 83200
    for (i, o) in [(256, 256), (512, 512), (128, 80)]:
        w = torch.nn.Parameter(torch.randn(o, i, device=dev) * 0.05)
        x = torch.randn(rows, i, device=dev).bfloat16().requires_grad_(True)
        g = torch.randn(rows, o, device=dev).bfloat16()
        for tuned in (True, False):
            opts = KernelOptions(tunableop=tuned)

            def layer():
                y = M._LinearReLU.apply(x, w, torch.bfloat16, False, False, False, None, opts)
                y.backward(g)
            res[f"layer_{i}x{o}_fwd_bwd_us_tuned{int(tuned)}"] = per_call_us(layer, 40)

            def fwd():
                M._LinearReLU.apply(x, w, torch.bfloat16, False, False, False, None, opts)
            res[f"layer_{i}x{o}_fwd_us_tuned{int(tuned)}"] = per_call_us(fwd, 40)
        wb = w.detach().bfloat16()
        xd = x.detach()
        res[f"wgrad_{i}x{o}_us"] = per_call_us(lambda: M._wgrad(g, xd), 40)
        res[f"addmm_act_{i}x{o}_us"] = per_call_us(
            lambda: torch._addmm_activation(M._zero_bias(o, torch.bfloat16, dev), xd, wb.t(), use_gelu=False), 40)
        res[f"mm_dgrad_{i}x{o}_us"] = per_call_us(lambda: g @ wb, 40)
        res[f"threshold_bwd_{i}x{o}_us"] = per_call_us(lambda: torch.ops.aten.threshold_backward(g, g, 0), 40)
        from avr_amd.wcache import cast_weight
        res[f"cast_weight_{i}x{o}_us"] = per_call_us(lambda: cast_weight(w, torch.bfloat16, False), 40)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
