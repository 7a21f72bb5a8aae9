"""Serial IR-render latency of one pose (default config 2) issued eagerly vs
replayed by avr_amd.graph.GraphedRender (stub network).  One JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


class Stub(torch.nn.Module):
    draws_no_device_rng = True

    def __init__(self, a, s):
        super().__init__()
        self.a, self.s = a, s

    def forward(self, *args, **kw):
        return self.a, self.s


def lat(fn, n=50):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / n


def main():
    dev = torch.device("cuda", 0)
    w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c2_meshrir_1024x256x512"]
    g = torch.Generator(device=dev).manual_seed(0)
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=dev, generator=g) * 0.1
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    r = AVRRender(Stub(attn, sig), **w.render)
    res = {"workload": w.name}
    with torch.no_grad():
        res["eager_ms"] = lat(lambda: r.render_ir(ro, tx))
        from avr_amd.graph import GraphedRender
        gr = GraphedRender(r)
        res["graph_ms"] = lat(lambda: gr.render_ir(ro, tx))
        res["eager_again_ms"] = lat(lambda: r.render_ir(ro, tx))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
