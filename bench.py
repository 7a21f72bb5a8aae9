"""Benchmark: MeshRIR single-listener render (config 2) through the IR.

One step = one pass of the hot path over one pose of synthetic input with the
network output already resident in HBM (stub network, as the reference's own
CPU timing does): ray generation + sampling (network inputs) -> weights ->
ray-reduction stream -> MFMA DFT + phase -> spectrum -> irfft IR.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

For N > 1 launch with torch.distributed.run (one process per GPU); each rank
renders its own poses (weak scaling, no data-path collective), rank 0 prints
one JSON line with the whole-job ray-samples/s.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender  # noqa: E402
from avr_amd import renderer as rmod  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


class StubNet(torch.nn.Module):
    def __init__(self, attn, signal):
        super().__init__()
        self.attn, self.signal = attn, signal

    def forward(self, pts, view, tx, dir_tx=None, ch_idx=None):
        return self.attn, self.signal


class KernelTimer:
    """HIP events around the ray-reduction kernel on the stream it runs on.

    Events are created up front (creating one inside the timed loop costs
    more host time than the render issues).  Also keeps each launch's delay
    tensor so the live window of every row, [delay, T-1-shift[s]) (the only
    signal elements the result depends on and the only ones the kernel
    reads), can be counted afterwards."""

    def __init__(self, n=0):
        self.pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                     for _ in range(n)]
        for a, b in self.pool:  # torch creates the HIP event at its first record
            a.record()
            b.record()
        torch.cuda.synchronize()
        self.used = 0
        self.rows = []
        self.n_split = None
        self.enabled = False

    def events(self, n_split=None, delay=None, shift=None):
        """(begin, end) raw hipEvent_t handles the library records around the
        ray-reduction launch on its stream (avr_render_core_fwd), or Nones."""
        if not self.enabled or self.used >= len(self.pool):
            return None, None
        self.n_split = n_split
        self.rows.append((delay, shift))
        a, b = self.pool[self.used]
        self.used += 1
        return a.cuda_event, b.cuda_event

    def mean_ms(self):
        ts = [a.elapsed_time(b) for a, b in self.pool[:self.used]]
        return sum(ts) / len(ts) if ts else float("nan")

    def mean_live_elements(self, T):
        """Average number of live signal elements per launch."""
        tot = 0.0
        for delay, shift in self.rows:
            lim = (T - 1 - shift.long()).clamp(min=0)
            tot += float((lim.view(1, 1, -1) - delay.long()).clamp(min=0).sum())
        return tot / max(1, len(self.rows))


def pmc_traffic(workload, dtype_name):
    """HBM bytes per launch of the reduction kernel from the newest committed
    rocprofv3 --pmc summary for this workload (tools/pmc_summary.py; the
    gfx950 FETCH_SIZE x2 correction applied there), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_*.json")))
    for path in reversed(files):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        for k, v in d["kernels"].items():
            if k.startswith("void ray_reduce_fwd_kernel<" + dtype_name):
                return v["hbm_bytes"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(w, budget_s=15.0):
    """Time the CPU oracle (op-for-op torch-CPU restatement of renderer_cpu.py)
    on this host's cores for a bounded sample of the same workload."""
    from oracle import avr_oracle as orc

    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(1)
    B, RS, T = w.batch, w.n_rays * w.n_samples, w.T
    attn = torch.rand(B, RS, 1, generator=g) * 2
    sig = torch.randn(B, RS, T, generator=g) * 0.1
    if w.signal_dtype == "float16":
        sig = sig.half()
    rays_o = torch.rand(B, 3, generator=g) * 4 - 2
    tx = torch.rand(B, 3, generator=g) * 4 - 2
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1) if w.with_dir_tx else None
    cfg = orc.RenderConfig.from_kwargs(**w.render)
    net = orc.StubNetwork(attn, sig)
    times = []
    t_start = time.time()
    while True:
        t0 = time.time()
        out = orc.render_spectrum(cfg, net, rays_o, tx, dtx)
        orc.spectrum_to_ir(out)
        times.append(time.time() - t0)
        if time.time() - t_start > budget_s or len(times) >= 20:
            break
    best = min(times)
    return {
        "value": w.ray_samples / best,
        "unit": "ray-samples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(times)} full poses of {w.name} (forward + irfft), best of {len(times)}; "
                  f"median {sorted(times)[len(times) // 2] * 1e3:.1f} ms/pose",
        "ms_per_pose": best * 1e3,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--poses", type=int, default=16,
                    help="distinct synthetic poses cycled over the steps")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams the independent per-pose renders are issued on "
                         "round-robin (1 = strictly serial)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    w = WORKLOADS[args.workload]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    dt = torch.float16 if w.signal_dtype == "float16" else torch.float32
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    attn = (torch.rand(B, R * S, 1, device=dev, generator=gen) * 2).to(dt)
    signal = (torch.randn(B, R * S, T, device=dev, generator=gen) * 0.1).to(dt)
    # a fixed set of listener/source poses, cycled: the live window of each
    # row (and so the bytes the reduction reads) depends on the geometry
    P = args.poses
    rays_o = torch.rand(P, B, 3, device=dev, generator=gen) * 4 - 2
    tx = torch.rand(P, B, 3, device=dev, generator=gen) * 4 - 2
    dtx = (torch.nn.functional.normalize(torch.randn(P, B, 3, device=dev, generator=gen), dim=-1)
           if w.with_dir_tx else [None] * P)
    renderer = AVRRender(StubNet(attn, signal), **w.render)
    timer = KernelTimer(args.steps)
    rmod.KERNEL_TIMER = timer
    pose = [0]

    def step():
        i = pose[0] % P
        pose[0] += 1
        with torch.no_grad():
            return renderer.render_ir(rays_o[i], tx[i], dtx[i])

    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(args.streams - 1)]

    def run(n, n_streams):
        for i in range(n):
            with torch.cuda.stream(streams[i % n_streams]):
                step()

    torch.manual_seed(rank)
    run(args.warmup, args.streams)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    # latency: one pose at a time on one stream (IR render ms/pose)
    n_lat = max(5, min(args.steps, 20))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_lat):
        step()
        torch.cuda.synchronize()
    latency_ms = (time.perf_counter() - t0) * 1e3 / n_lat

    # roofline phase: K launches on ONE stream with HIP events around the
    # dominant kernel on its stream, so no other kernel overlaps it and the
    # events bracket exactly the kernel (a rocprofv3 trace of this command
    # gives the same average; events inside the 2-stream phase would also
    # count the wait for the other stream and slow its issue down)
    timer.enabled = True
    run(args.steps, 1)
    torch.cuda.synchronize()
    timer.enabled = False

    # throughput (the reported value): K independent single-pose renders
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, args.streams)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed * 1e3 / args.steps
    total_rs = world * w.ray_samples * args.steps
    value = total_rs / elapsed

    # roofline for the dominant kernel (ray-reduction stream)
    k_ms = timer.mean_ms()
    es = 2 if dt == torch.float16 else 4
    n_split = timer.n_split or 1
    # algorithmic bytes: the live signal elements (each read once), w + delay
    # (8 B per ray-sample), the fp32 partials written; the dense tensor is
    # reported beside it
    live = timer.mean_live_elements(T)
    alg_bytes = live * es + w.ray_samples * 8 + n_split * B * S * T * 4
    dense_bytes = w.ray_samples * (T * es + 8) + n_split * B * S * T * 4
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9

    traffic, traffic_src = pmc_traffic(w.name, "__half" if dt == torch.float16 else "float")

    result = {
        "metric": "ray-samples/sec/GPU (1024 rays×256 samp×512 freq) + IR render ms/pose",
        "value": value,
        "unit": "ray-samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "ir_render_ms_per_pose": latency_ms / B,
        "host_issue_ms_per_step": t_issue * 1e3 / args.steps,
        "streams": args.streams,
        "per_gpu_value": value / world,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if dt == torch.float32 else "f16-storage/f32-math",
        "data": "synthetic (stub network, outputs resident in HBM; seeded torch RNG)",
        "config": {"workload": w.name, "rays": R, "samples": S, "T": T, "freq_bins": w.F,
                   "poses_per_step": B, "distinct_poses": P, "parallelism": f"poses x{world} (no data-path collective)",
                   "pipelining": f"{args.streams} HIP streams, consecutive poses round-robin"},
        "roofline": {
            "kernel": "ray_reduce_fwd_kernel",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "alg_bytes_per_launch": alg_bytes,
            "dense_bytes_per_launch": dense_bytes,
            "live_fraction": live / (w.ray_samples * T),
            "avg_launch_ms": k_ms,
            "measured": "HIP events around each launch, roofline phase of K steps on one stream",
        },

    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(w, args.cpu_budget)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
