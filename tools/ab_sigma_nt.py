"""Interleaved A/B of the h1 stores of `sigma_meshrir_h1` at config 2 (fp16):
streaming (nontemporal, the default) against plain stores, timed together
with the width-512 layer that reads h1 next, since the stores' cache policy
matters to that reader.  Uses the shape-probe library
(`make -C avr_amd/csrc shapes`; AVR_SIGMA_NT_PROBE).

    python tools/ab_sigma_nt.py [--rounds 5] [--iters 20]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from avr_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("AVR_AB_LIB") or os.path.join(ROOT, "tools", "_lib", "libavr_shapes.so")
from avr_amd import sigma  # noqa: E402
from avr_amd.model import _enable_tuned_gemms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    N, S = 262144, 256
    v = sigma.MESHRIR_H1
    ws = [torch.randn(M, K, device=dev) * np.sqrt(2.0 / K) for M, K, _, _ in sigma.SCHEDULE[v]]
    packed = sigma.pack_layers(v, ws, torch.float16)
    inputs = [(torch.rand(N, 40, device=dev).half(), 1)]
    bias = torch.randn(N // S, 512, device=dev) * 0.1
    W2 = (torch.randn(512, 512, device=dev) / 512 ** 0.5).half()
    b2 = torch.zeros(512, device=dev).half()
    _enable_tuned_gemms(dev)

    def step():
        _, h1 = sigma.sigma_fwd(v, packed, N, inputs, [], 512, 0.01, bias=bias, bias_div=S)
        return torch._addmm_activation(b2, h1, W2.t())

    modes = {"nt": "1", "plain": "0"}
    res = {m: [] for m in modes}
    outs = {}
    with torch.no_grad():
        for m, f in modes.items():
            os.environ["AVR_SIGMA_NT_PROBE"] = f
            outs[m] = step().clone()
        print("outputs equal:", bool(torch.equal(outs["nt"], outs["plain"])), flush=True)
        for _ in range(a.rounds):
            for m, f in modes.items():
                os.environ["AVR_SIGMA_NT_PROBE"] = f
                for _ in range(5):
                    step()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    step()
                e1.record()
                e1.synchronize()
                res[m].append(e0.elapsed_time(e1) / a.iters * 1e3)
    for m in modes:
        r = sorted(res[m])
        print(f"{m}: median {r[len(r) // 2]:.1f} us, min {r[0]:.1f} (sigma h1 + 512x512 layer)", flush=True)


if __name__ == "__main__":
    main()
