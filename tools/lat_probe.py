"""Where the serial IR-render latency of a graph replay goes (config 2, stub
network, host poses as in bench.py): GPU chain time by events, host time of
the render_ir call, and the per-pose latency under different ways of
waiting for the result.  One JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from avr_amd import AVRRender  # noqa: E402
from avr_amd.graph import GraphedRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


class Stub(torch.nn.Module):
    draws_no_device_rng = True

    def __init__(self, a, s):
        super().__init__()
        self.a, self.s = a, s

    def forward(self, *args, **kw):
        return self.a, self.s


def main():
    dev = torch.device("cuda", 0)
    w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c2_meshrir_1024x256x512"]
    g = torch.Generator(device=dev).manual_seed(0)
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=dev, generator=g) * 0.1
    ro = (torch.rand(B, 3, generator=torch.Generator().manual_seed(1)) * 4 - 2)
    tx = (torch.rand(B, 3, generator=torch.Generator().manual_seed(2)) * 4 - 2)
    r = AVRRender(Stub(attn, sig), **w.render)
    gr = GraphedRender(r)
    n = 200
    res = {"workload": w.name}
    with torch.no_grad():
        for _ in range(gr.ring + 5):
            gr.render_ir(ro, tx)
        torch.cuda.synchronize()

        # GPU time of one replay (events on the stream around the call)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        gpu = []
        for _ in range(50):
            e0.record()
            gr.render_ir(ro, tx)
            e1.record()
            e1.synchronize()
            gpu.append(e0.elapsed_time(e1))
        gpu.sort()
        res["gpu_chain_ms_median"] = gpu[len(gpu) // 2]

        # host time of the call itself (no wait)
        host = []
        for _ in range(50):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gr.render_ir(ro, tx)
            host.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        host.sort()
        res["host_call_ms_median"] = host[len(host) // 2]

        # pieces of the call: the jitter draw, the pose staging, the replay
        key = next(iter(gr._graphs))
        inst = gr._graphs[key][0][0]
        parts = {"rand": [], "stage": [], "replay": [], "record": []}
        for _ in range(50):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            torch.rand(int(r.n_azi) + int(r.n_ele), out=inst.jit_h)
            t1 = time.perf_counter()
            inst.pose_h[:3].copy_(ro.reshape(-1))
            inst.pose_h[3:6].copy_(tx.reshape(-1))
            t2 = time.perf_counter()
            inst.graph.replay()
            t3 = time.perf_counter()
            inst.done.record()
            t4 = time.perf_counter()
            for k, a, b in (("rand", t0, t1), ("stage", t1, t2), ("replay", t2, t3), ("record", t3, t4)):
                parts[k].append((b - a) * 1e3)
        torch.cuda.synchronize()
        for k, v in parts.items():
            v.sort()
            res[f"host_{k}_ms_median"] = v[len(v) // 2]

        def lat(wait):
            for _ in range(10):
                gr.render_ir(ro, tx)
                wait()
            t0 = time.perf_counter()
            for _ in range(n):
                gr.render_ir(ro, tx)
                wait()
            return (time.perf_counter() - t0) * 1e3 / n

        ev = torch.cuda.Event()

        def ev_sync():
            ev.record()
            ev.synchronize()

        def ev_spin():
            ev.record()
            while not ev.query():
                pass

        res["lat_device_sync_ms"] = lat(torch.cuda.synchronize)
        res["lat_event_sync_ms"] = lat(ev_sync)
        res["lat_event_spin_ms"] = lat(ev_spin)
        res["lat_device_sync_ms_again"] = lat(torch.cuda.synchronize)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
