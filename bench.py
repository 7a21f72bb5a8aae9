"""Benchmark: the acoustic volume render path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode MODE] [--workload NAME]

Modes (a "step" is one pass of the hot path over one unit of synthetic input):

* `pose` (default, the BASELINE metric): MeshRIR single-listener render,
  config 2 (1024 rays x 256 samples x 512 bins).  One step = one pose through
  the IR with the network output already resident in HBM (stub network, as
  the reference's own CPU timing does): ray generation + sampling -> weights
  -> ray-reduction stream -> MFMA DFT + phase -> spectrum -> irfft IR.  With
  N ranks every rank renders its own poses (weak scaling, no data-path
  collective: poses are independent).
* `ray-shard`: config 5 (4096 x 512 x 2048 bins, fp16 signal), ONE pose whose
  rays are split over the N ranks (avr_amd.parallel.RayShardedRender) with the
  spectrum all-reduce over RCCL inside the timed region, then the IR (strong
  scaling: the pose is fixed, each rank holds 17.2 GB / N of signal).
* `ddp-train`: config 4 (RAF-Empty, 4 poses per rank), the full training step
  (avr_runner_ddp.py:131-137 body: AVRModel_complex -> render -> criterion ->
  backward with DDP's bucketed RCCL gradient all-reduce -> clip + Adam ->
  scheduler) (weak scaling).

`--gpus N` with N > 1 outside torchrun re-launches this script under
`torch.distributed.run` (one process per GPU) before any GPU call; under
torchrun the world size comes from the environment and must equal --gpus.
Rank 0 prints ONE JSON line; `value` is the whole-job throughput = units all
ranks processed / max-over-ranks time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "ray-samples/sec/GPU (1024 rays×256 samp×512 freq) + IR render ms/pose"
MODES = {  # mode -> default workload (avr_amd.workloads.WORKLOADS)
    "pose": "c2_meshrir_1024x256x512",
    "ray-shard": "c5_simu_4096x512x2048",
    "ddp-train": "c4_raf_empty_b4_per_gpu",
}


class StubNet(torch.nn.Module):
    draws_no_device_rng = True  # avr_amd.graph: replay without torch's RNG prologue

    def __init__(self, attn, signal):
        super().__init__()
        self.attn, self.signal = attn, signal

    def forward(self, pts, view, tx, dir_tx=None, ch_idx=None):
        return self.attn, self.signal


class KernelTimer:
    """HIP events around the ray-reduction kernel on the stream it runs on
    (set as `AVRRender.kernel_timer`).

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

    def head_events(self, delay=None, shift=None, K=0):
        """(begin, end) torch events to record around the rounding-exact head's
        launch (FusedHeadCore, network mode: the fused head replaces the ray
        reduction), or Nones.  Keeps the launch's delays for the live count."""
        if not self.enabled:
            return None, None
        if not hasattr(self, "head_pool"):
            self.head_pool, self.head_rows, self.head_K = [], [], K
        if len(self.head_pool) >= len(self.pool):
            return None, None
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        self.head_pool.append(ev)
        self.head_rows.append((delay, shift))
        self.head_K = K
        return ev

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


# ----------------------------------------------------------------------------
# launcher (no GPU call before the ranks exist)
# ----------------------------------------------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE under torchrun, else 1")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", default="pose", choices=sorted(MODES))
    ap.add_argument("--workload", default=None, help="default: the mode's workload")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--network", action="store_true",
                    help="ray-shard mode: render through the reference network (AVRModel, avr_simu.yml "
                         "model block, random init, --mlp-dtype MLPs, fused rounding-exact head) instead of "
                         "the stub's resident outputs")
    ap.add_argument("--no-network", action="store_true",
                    help="pose mode: skip the config-2 inference through the reference network")
    ap.add_argument("--poses", type=int, default=16,
                    help="distinct synthetic poses cycled over the steps")
    ap.add_argument("--graph-ring", type=int, default=12,
                    help="captured graph instances per stream (GraphedRender ring)")
    ap.add_argument("--streams", type=int, default=2,
                    help="pose mode: HIP streams the independent per-pose renders are issued on "
                         "round-robin, each with its own signal buffer (1 = strictly serial; "
                         "on MI355X 2, 3 and 4 streams measure the same within 1%%)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="ray-shard mode on one GPU: render rank 0's shard of an N-rank job (its rays only, "
                         "no collective): the per-rank time an N-GPU run would see")
    ap.add_argument("--mlp-dtype", default="bf16", choices=["bf16", "fp16", "fp32"],
                    help="ddp-train mode: MLP compute dtype")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="rehearsal of the N-rank path on ONE GPU: every rank on cuda:0, "
                         "process group over gloo (RCCL needs one GPU per rank); the numbers "
                         "are not a scaling measurement")
    args = ap.parse_args(argv)
    if args.workload is None:
        args.workload = MODES[args.mode]
    return args


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_command(n, argv, port, script=None):
    """The torch.distributed.run command that starts n ranks of this script."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}",
            script or os.path.abspath(__file__), *argv]


def resolve_world(args, env=None, device_count=None):
    """('launch', n) to start n ranks, ('run', world) to run as one of them.

    Raises SystemExit with a clear message when the request cannot be met:
    --gpus disagreeing with a torchrun world, or more GPUs than visible."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} "
                             "(launch with --nproc-per-node equal to --gpus)")
        return "run", world
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if n == 1:
        return "run", 1
    if args.oversubscribe:
        return "launch", n
    # counting devices does not initialise the GPU on this image
    have = torch.cuda.device_count() if device_count is None else device_count
    if have < n:
        raise SystemExit(f"bench.py: --gpus {n} requested but only {have} GPU(s) visible")
    return "launch", n


def timed(run, world, dev):
    """Barrier + synchronize on both sides of run(); max over ranks (s).
    (`dev` may be the CPU: the gloo tests of this logic.)"""
    import torch.distributed as dist

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run()
    t_issue = time.perf_counter() - t0
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, t_issue


def whole_job_rate(units_per_rank, world, steps, elapsed_max):
    """value: units every rank processed over the slowest rank's time."""
    return units_per_rank * world * steps / elapsed_max


# ----------------------------------------------------------------------------
# measurement helpers
# ----------------------------------------------------------------------------
def pmc_traffic(workload, dtype_name):
    """HBM bytes per launch of the reduction kernel from the newest committed
    rocprofv3 --pmc summary for this workload (tools/pmc_summary.py; the
    gfx950 FETCH_SIZE x2 correction applied there), or None."""
    import glob

    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_*.json")):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        for k, v in d["kernels"].items():
            if k.startswith("void ray_reduce_fwd_kernel<" + dtype_name):
                # newest by the round and time recorded in the summary, not by file name
                key = (int(d.get("round", 0)), str(d.get("measured_at", "")))
                if best is None or key > best[0]:
                    best = (key, v["hbm_bytes"], os.path.relpath(path, ROOT))
    return (best[1], best[2]) if best else (None, None)


def roofline(w, timer, dt):
    """Roofline object for the ray-reduction kernel from the live HIP events."""
    B, S, T = w.batch, w.n_samples, w.T
    k_ms = timer.mean_ms()
    es = 2 if dt == torch.float16 else 4
    n_split = timer.n_split or 1
    # algorithmic bytes: the live signal elements (each read once), w + delay
    # (8 B per ray-sample), the fp32 partials written; the dense tensor is
    # reported beside it (SURVEY.md §8d's basis; the kernel never reads the
    # masked elements, so only the live basis bounds it)
    live = timer.mean_live_elements(T)
    # ray-samples one launch covers (this rank's shard in ray-shard mode)
    rows = timer.rows[0][0].numel() if timer.rows else w.ray_samples
    alg_bytes = live * es + rows * 8 + n_split * B * S * T * 4
    dense_bytes = rows * (T * es + 8) + n_split * B * S * T * 4
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(w.name, "__half" if dt == torch.float16 else "float")
    return {
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
        "dense_frac": dense_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "live_fraction": live / (rows * T) if rows else 0.0,
        "avg_launch_ms": k_ms,
        "measured": "HIP events around each launch, roofline phase of K steps on one stream",
    }


MFMA_PEAK_TFS_16 = 2500.0  # MI355X_MICROARCH.md: fp16 / bf16 dense MFMA, ~2.5 PF/s


def head_roofline(w, timer):
    """Roofline object for the rounding-exact head (network mode): algorithmic
    FLOPs = 2 K x the live (ray-sample, t) elements of the launch (the
    [delay, T-1-shift[s]) windows, the only products the render uses), over
    the launch's HIP-event duration; against the dense 16-bit MFMA peak."""
    pool = getattr(timer, "head_pool", [])
    if not pool:
        return None
    ts = [a.elapsed_time(b) for a, b in pool]
    k_ms = sum(ts) / len(ts)
    T, K = w.T, timer.head_K
    live = 0.0
    for delay, shift in timer.head_rows:
        lim = (T - 1 - shift.long()).clamp(min=0)
        live += float((lim.view(1, 1, -1) - delay.long()).clamp(min=0).sum())
    live /= len(timer.head_rows)
    rows = timer.head_rows[0][0].numel()
    flops = 2.0 * K * live
    achieved = flops / (k_ms * 1e-3) / 1e12
    traffic, src = None, None
    for path in sorted(glob_profiles("r*_pmc_c5_network_fp16.json")):
        d = json.load(open(path))
        for k, v in d.items():
            if k.startswith("head_exact_kernel<__half") and w.name.startswith("c5_"):
                traffic = v["derived"]["hbm_read_bytes"] + v["derived"]["hbm_write_bytes"]
                src = os.path.relpath(path, ROOT)
    return {
        "kernel": "head_exact_kernel",
        "bound": "mfma",
        "achieved": achieved,
        "peak": MFMA_PEAK_TFS_16,
        "unit": "TFLOP/s",
        "frac": achieved / MFMA_PEAK_TFS_16,
        "traffic": traffic,
        "traffic_source": src,
        "alg_flops_per_launch": flops,
        "dense_flops_per_launch": 2.0 * K * rows * T,
        "live_fraction": live / (rows * T) if rows else 0.0,
        "avg_launch_ms": k_ms,
        "measured": "HIP events around each head launch on its stream, the timed steps",
    }


def adam_roofline(events, n_params):
    """Roofline object for the training step's optimizer pass (avr_adam_step:
    clipped, sanitised Adam over every fp32 parameter; p, g, m, v read, p, m,
    v written: 28 algorithmic bytes per parameter) from HIP events around its
    launches."""
    if not events:
        return None
    ts = [a.elapsed_time(b) for a, b in events]
    k_ms = sum(ts) / len(ts)
    alg = 28.0 * n_params
    achieved = alg / (k_ms * 1e-3) / 1e9
    return {
        "kernel": "adam_kernel",
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": None,
        "alg_bytes_per_launch": alg,
        "params": n_params,
        "avg_launch_ms": k_ms,
        "measured": "HIP events around the optimizer's Adam launches (one per step), a phase of K steps "
                    "before the timed region",
    }


def glob_profiles(pattern):
    import glob

    return glob.glob(os.path.join(ROOT, "profiles", pattern))


def cpu_baseline(w, budget_s=15.0, mode="pose"):
    """Time the CPU oracle (op-for-op torch-CPU restatement of renderer_cpu.py)
    on this host's cores for a bounded sample of the mode's workload:

    * pose: full poses of the workload, forward + irfft;
    * ray-shard: ONE rank's share of the pose (config 5 on the
      CPU as a 1/8 ray shard): a sphere with about R/8 rays, all samples,
      the full T, forward + irfft (the whole pose does not fit host RAM);
    * ddp-train: the render core's forward + backward (reference autograd)
      at the per-rank shape (the CPU has no hash-grid/MLP network to time).
    `value` is ray-samples per second in every mode."""
    from oracle import avr_oracle as orc

    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(1)
    sample = w
    if mode == "ray-shard":
        n_ele = w.render["n_ele"]
        n_azi = max(1, round((w.n_rays / 8 - 2) / n_ele))
        sample = w.replace(n_azi=n_azi)
    B, RS, T = sample.batch, sample.n_rays * sample.n_samples, sample.T
    attn = torch.rand(B, RS, 1, generator=g) * 2
    sig = torch.randn(B, RS, T, generator=g) * 0.1
    if sample.signal_dtype == "float16":
        sig = sig.half()
    rays_o = torch.rand(B, 3, generator=g) * 4 - 2
    tx = torch.rand(B, 3, generator=g) * 4 - 2
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, generator=g), dim=-1) if sample.with_dir_tx else None
    cfg = orc.RenderConfig.from_kwargs(**sample.render)
    train = mode == "ddp-train"
    if train:
        attn.requires_grad_(True)
        sig.requires_grad_(True)
        probe = torch.randn(B, sample.F, 2, generator=g)
    net = orc.StubNetwork(attn, sig)
    times = []
    t_start = time.time()
    warm = True  # the first pass (allocator, thread pool, FFT plans) is not timed
    while True:
        t0 = time.time()
        if train:
            out = orc.render_spectrum(cfg, net, rays_o, tx, dtx)
            (out * probe).sum().backward()
            attn.grad = sig.grad = None
        else:
            with torch.no_grad():
                out = orc.render_spectrum(cfg, net, rays_o, tx, dtx)
                orc.spectrum_to_ir(out)
        if not warm:
            times.append(time.time() - t0)
        warm = False
        del out
        if times and (time.time() - t_start > budget_s or len(times) >= 20):
            break
    best = min(times)
    what = {"pose": "full poses of {n} (forward + irfft)",
            "ray-shard": "1/8 ray shards of {n}: {r} rays ({a}x{e}+2) x {s} samples x T={t} (forward + irfft)",
            "ddp-train": "render-core forward + backward (reference autograd) of {n}, {b} poses"}[mode]
    what = what.format(n=w.name, r=sample.n_rays, a=sample.render["n_azi"], e=sample.render["n_ele"],
                       s=sample.n_samples, t=T, b=B)
    return {
        "value": sample.ray_samples / best,
        "unit": "ray-samples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(times)} x {what}; best of {len(times)}, "
                  f"median {sorted(times)[len(times) // 2] * 1e3:.1f} ms",
        "ms_per_pose": best * 1e3,
    }


def cpu_leg_threads():
    """Host threads for the CPU leg: the process's own setting, raised to the
    box's per-GPU CPU share (16) when a launcher left it at 1 (torchrun sets
    OMP_NUM_THREADS=1 when the environment has none); AVR_CPU_THREADS
    overrides."""
    want = int(os.environ.get("AVR_CPU_THREADS", "0"))
    return want if want > 0 else max(torch.get_num_threads(), min(16, os.cpu_count() or 1))


def attach_cpu_baseline(result, args, w, world, rank):
    """The CPU leg in the same run at every world size (BASELINE.json
    north_star: renderer_cpu.py timed beside the 1/2/4/8-GPU numbers): rank 0
    times the oracle after the timed region and the other ranks wait for it
    at a barrier, so no rank's GPU work overlaps it."""
    if rank == 0 and not args.no_cpu_baseline:
        prev = torch.get_num_threads()
        torch.set_num_threads(cpu_leg_threads())
        try:
            result["cpu_baseline"] = cpu_baseline(w, args.cpu_budget, args.mode)
        finally:
            torch.set_num_threads(prev)
        if world > 1:
            result["cpu_baseline"]["note"] = (f"timed on rank 0's host after the {world}-rank timed region, "
                                              "the other ranks idle at a barrier")
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def network_inference(w, dev, steps=20, warmup=3):
    """Config-2 inference through the reference's own network, not the stub:
    AVRModel with the avr_meshrir.yml `model:` block (random init), MLPs in
    fp16 as tcnn runs them (model.py:21-31), one pose per step, no grad,
    through the IR.  The default path: level-major hash grids, fused sigma
    networks and first signal layer (csrc/sigma.hip), hipBLASLt for the two
    512x512 signal layers, the fused signal head (csrc/head.hip) and the
    render tail.  Reported beside `value`, which stays SURVEY §8(d)'s
    stub-network metric."""
    from avr_amd import AVRRender, spectrum_to_ir
    from avr_amd.model import AVRModel
    from avr_amd.workloads import MESHRIR_MODEL

    torch.manual_seed(0)
    model = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=w.T), mlp_dtype=torch.float16).to(dev)
    r = AVRRender(model, **w.render)
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2

    def step():
        with torch.no_grad():
            return spectrum_to_ir(r(ro, tx))

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / steps
    return {
        "network": "AVRModel (avr_meshrir.yml model block, random init), fp16 MLPs (tcnn precision)",
        "path": "level-major hash grids + fused sigma networks + hipBLASLt 512x512 layers (TunableOp-selected solution, avr_amd/tunableop_gfx950.csv) + fused signal head "
                "+ render + irfft",
        "ms_per_pose": ms,
        "ray_samples_per_s": w.ray_samples / (ms * 1e-3),
        "steps": steps,
    }


def _poses(w, P, dev, gen):
    rays_o = torch.rand(P, w.batch, 3, device=dev, generator=gen) * 4 - 2
    tx = torch.rand(P, w.batch, 3, device=dev, generator=gen) * 4 - 2
    dtx = (torch.nn.functional.normalize(torch.randn(P, w.batch, 3, device=dev, generator=gen), dim=-1)
           if w.with_dir_tx else [None] * P)
    return rays_o, tx, dtx


def _base_result(args, w, world, value, elapsed, dtype):
    return {
        "metric": METRIC,
        "value": value,
        "unit": "ray-samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "per_gpu_value": value / world,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (stub network, outputs resident in HBM; seeded torch RNG)",
    }


# ----------------------------------------------------------------------------
# modes
# ----------------------------------------------------------------------------
def bench_pose(args, w, world, rank, dev):
    from avr_amd import AVRRender

    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    dt = torch.float16 if w.signal_dtype == "float16" else torch.float32
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    n_streams = max(1, args.streams)
    # one network output per stream, so concurrent renders never share
    # addresses (no cross-stream cache reuse can inflate the rate)
    renderers = []

    def add_renderer():
        attn = (torch.rand(B, R * S, 1, device=dev, generator=gen) * 2).to(dt)
        signal = (torch.randn(B, R * S, T, device=dev, generator=gen) * 0.1).to(dt)
        renderers.append(AVRRender(StubNet(attn, signal), **w.render))

    # a fixed set of listener/source poses, cycled: the live window of each
    # row (and so the bytes the reduction reads) depends on the geometry.  The
    # poses are drawn after exactly two network outputs whatever the stream
    # count, so every --streams setting renders the same poses (the set
    # earlier rounds measured at 2 streams)
    add_renderer()
    add_renderer()
    P = args.poses
    rays_o, tx, dtx = _poses(w, P, dev, gen)
    while len(renderers) < n_streams:
        add_renderer()
    del renderers[n_streams:]
    timer = KernelTimer(args.steps)
    renderers[0].kernel_timer = timer
    pose = [0]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_streams - 1)]

    def step(k):
        i = pose[0] % P
        pose[0] += 1
        with torch.no_grad():
            return renderers[k].render_ir(rays_o[i], tx[i], dtx[i])

    def run(n, ns):
        for i in range(n):
            with torch.cuda.stream(streams[i % ns]):
                step(i % ns)

    torch.manual_seed(rank)
    run(args.warmup, n_streams)
    torch.cuda.synchronize()

    # latency: one pose at a time on one stream (IR render ms/pose), issued
    # eagerly and replayed from a HIP graph (avr_amd.graph.GraphedRender:
    # same kernels and results bit for bit, no per-launch host work)
    n_lat = max(5, min(args.steps, 20))

    def latency(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_lat):
            fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n_lat

    latency_eager_ms = latency(lambda: step(0))
    from avr_amd.graph import GraphedRender

    graphed = GraphedRender(renderers[0], ring=args.graph_ring)
    # poses handed over from the host, as a data loader yields them
    # (avr_runner.py:168): staged in the replay's pinned buffer, no copy
    ro_h, tx_h = rays_o.cpu(), tx.cpu()
    dtx_h = [None if d is None else d.cpu() for d in dtx]

    def step_graph():
        i = pose[0] % P
        pose[0] += 1
        with torch.no_grad():
            return graphed.render_ir(ro_h[i], tx_h[i], dtx_h[i])

    for _ in range(graphed.ring + 2):  # captures
        step_graph()
    latency_ms = latency(step_graph)

    # roofline phase: K launches on ONE stream with HIP events around the
    # dominant kernel on its stream, so no other kernel overlaps it and the
    # events bracket exactly the kernel (a rocprofv3 trace of this command
    # gives the same average)
    timer.enabled = True
    run(args.steps, 1)
    torch.cuda.synchronize()
    timer.enabled = False

    # throughput: K independent single-pose renders on 2 streams, issued
    # eagerly (the reported value) and, as a second measurement, replayed
    # from each stream's HIP graph ring (the same kernels and results,
    # tests/test_gpu_graph.py; host poses staged in pinned memory).  Since
    # round 3 the eager issue (~75 us of host work per pose) no longer gates
    # a ~120 us pose, and it keeps each stream's kernels back to back, while
    # consecutive graph replays on one stream leave 15-23 us between them
    # (kernel trace): eager measured 0.1186-0.1226 against
    # 0.1210-0.1308 ms per pose for the replays over 4 runs of the driver's
    # command (tools/gpu_eager_graph.sh)
    graphs = [graphed] + [GraphedRender(rr, ring=args.graph_ring) for rr in renderers[1:]]

    def run_graph(n, ns):
        for i in range(n):
            k = i % ns
            with torch.cuda.stream(streams[k]):
                j = pose[0] % P
                pose[0] += 1
                with torch.no_grad():
                    graphs[k].render_ir(ro_h[j], tx_h[j], dtx_h[j])

    run_graph(max(args.warmup, (graphed.ring + 2) * n_streams), n_streams)  # captures + warm replays
    torch.cuda.synchronize()
    elapsed, t_issue = timed(lambda: run(args.steps, n_streams), world, dev)
    elapsed_graph, t_issue_graph = timed(lambda: run_graph(args.steps, n_streams), world, dev)
    value = whole_job_rate(w.ray_samples, world, args.steps, elapsed)
    res = _base_result(args, w, world, value, elapsed, "f32" if dt == torch.float32 else "f16-storage/f32-math")
    res.update({
        "ir_render_ms_per_pose": latency_ms / B,
        "ir_render_path": "HIP-graph replay (avr_amd.graph.GraphedRender), host poses, synchronized per pose",
        "ir_render_ms_per_pose_eager": latency_eager_ms / B,
        "host_issue_ms_per_step": t_issue * 1e3 / args.steps,
        "throughput_path": "eager issue, 2 HIP streams round-robin (one ctypes render-core call per pose)",
        "ms_per_step_graph": elapsed_graph * 1e3 / args.steps,
        "host_issue_ms_per_step_graph": t_issue_graph * 1e3 / args.steps,
        "streams": n_streams,
        "config": {"workload": w.name, "mode": "pose", "rays": R, "samples": S, "T": T, "freq_bins": w.F,
                   "poses_per_step": B, "distinct_poses": P,
                   "parallelism": f"poses x{world} (no data-path collective)",
                   "pipelining": f"{n_streams} HIP streams, consecutive poses round-robin, "
                                 "one signal buffer and one graph ring per stream"},
        "roofline": roofline(w, timer, dt),
    })
    return res


def bench_ray_shard(args, w, world, rank, dev):
    from avr_amd import AVRRender, spectrum_to_ir
    from avr_amd.parallel import RayShardedRender, shard_range

    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    dt = torch.float16 if w.signal_dtype == "float16" else torch.float32
    shard_of = args.shard_of if args.shard_of > 1 else 0
    if shard_of and world != 1:
        raise SystemExit("--shard-of measures one rank's shard on a single GPU (--gpus 1)")
    r0, r1 = shard_range(R, rank, shard_of or world)
    Rl = r1 - r0
    if args.network:
        # the reference network of config 5 (avr_simu.yml), the same random
        # weights on every rank; each rank evaluates it on its own rays only
        from avr_amd.model import AVRModel
        from avr_amd.workloads import SIMU_MODEL
        mlp_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.mlp_dtype]
        torch.manual_seed(0)
        net = AVRModel(dict(SIMU_MODEL, signal_output_dim=T), mlp_dtype=mlp_dtype).to(dev)
    else:
        gen = torch.Generator(device=dev).manual_seed(1234 + rank)
        attn = (torch.rand(B, Rl * S, 1, device=dev, generator=gen) * 2).to(dt)
        signal = (torch.randn(B, Rl * S, T, device=dev, generator=gen) * 0.1).to(dt)
        net = StubNet(attn, signal)
    # every rank renders the same poses (one pose, its rays split)
    pg = torch.Generator(device=dev).manual_seed(4321)
    P = args.poses
    rays_o, tx, dtx = _poses(w, P, dev, pg)
    renderer = AVRRender(net, **w.render).to(dev)
    timer = KernelTimer(args.steps)
    renderer.kernel_timer = timer
    sharded = RayShardedRender(renderer, shard=(0, shard_of) if shard_of else None)
    pose = [0]

    def step():
        i = pose[0] % P
        pose[0] += 1
        with torch.no_grad():
            out = sharded(rays_o[i], tx[i], dtx[i])
            return out, spectrum_to_ir(out)

    def run(n):
        for _ in range(n):
            step()

    torch.manual_seed(7)  # same CPU jitter stream on every rank
    run(args.warmup)
    torch.cuda.synchronize()
    timer.enabled = True
    run(args.steps)
    torch.cuda.synchronize()
    timer.enabled = False
    elapsed, t_issue = timed(lambda: run(args.steps), world, dev)
    if shard_of:  # this shard's ray-samples per second (one rank's rate)
        value = whole_job_rate(B * Rl * S, 1, args.steps, elapsed)
    else:
        value = whole_job_rate(w.ray_samples, 1, args.steps, elapsed)  # one pose per step, all ranks
    res = _base_result(args, w, world, value, elapsed, "f32" if dt == torch.float32 else "f16-storage/f32-math")
    # with the network the fused head replaces the ray reduction: the head's
    # own events (FusedHeadCore, rounding-exact 16-bit head)
    rf = roofline(w, timer, dt) if not args.network else head_roofline(w, timer)
    if args.network:
        res["dtype"] = args.mlp_dtype + " MLP / f32 render"
        res["data"] = "synthetic poses; AVRModel (avr_simu.yml model block), random init, evaluated per ray shard"
    res.update({
        "scaling": "strong",
        "ir_render_ms_per_pose": elapsed * 1e3 / args.steps,
        "host_issue_ms_per_step": t_issue * 1e3 / args.steps,
        "config": {"workload": w.name, "mode": "ray-shard", "rays": R, "rays_per_rank": Rl, "samples": S,
                   "T": T, "freq_bins": w.F, "poses_per_step": B,
                   "parallelism": (f"rank 0's shard of a {shard_of}-rank ray split on one GPU, no collective "
                                   f"(the per-rank work of --gpus {shard_of}; value = this shard's ray-samples/s)"
                                   if shard_of else
                                   f"rays x{world}, one RCCL all-reduce of the [B,F,2] spectrum per pose"),
                   "network": "AVRModel (avr_simu.yml)" if args.network else "stub (outputs resident in HBM)"},
        "roofline": rf,
    })
    return res


def bench_ddp_train(args, w, world, rank, dev):
    from avr_amd import AVRRender
    from avr_amd.model import AVRModel_complex
    from avr_amd.parallel import ddp
    from avr_amd.training import TrainStep
    from avr_amd.workloads import RAF_MODEL

    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    mlp_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.mlp_dtype]
    torch.manual_seed(0)  # identical initial weights on every rank (DDP also broadcasts them)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=T), mlp_dtype=mlp_dtype).to(dev)
    r = AVRRender(model, **w.render).to(dev)
    net = ddp(r, dev) if world > 1 else r
    # RAF training config (config_files/avr_raf_*.yml:24-40)
    train_cfg = dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5,
                     spec_loss_weight=1, amplitude_loss_weight=1, angle_loss_weight=1,
                     time_loss_weight=20, energy_loss_weight=3, multistft_loss_weight=2)
    ts = TrainStep(net, train_cfg, w.render)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)  # each rank its own pose shard
    P = max(1, min(args.poses, 4))
    rays_o, tx, dtx = _poses(w, P, dev, g)
    tt = torch.arange(T, device=dev)
    targets = [torch.fft.rfft(torch.randn(B, T, device=dev, generator=g) * torch.exp(-tt / (0.15 * T)) * 0.05)
               for _ in range(P)]
    it = [0]

    def step():
        i = it[0] % P
        it[0] += 1
        ts(targets[i], rays_o[i], tx[i], dtx[i])

    def run(n):
        for _ in range(n):
            step()

    torch.manual_seed(rank)
    run(args.warmup)
    torch.cuda.synchronize()
    # roofline phase: HIP events around the optimizer's Adam launches (the
    # step's largest single kernel, HBM-bound), then the timed region
    pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    used = []
    ts.adam_events = lambda: used.append(pool[len(used)]) or used[-1] if len(used) < len(pool) else None
    run(args.steps)
    torch.cuda.synchronize()
    ts.adam_events = None
    elapsed, t_issue = timed(lambda: run(args.steps), world, dev)
    value = whole_job_rate(w.ray_samples, world, args.steps, elapsed)
    n_params = sum(p.numel() for p in r.parameters())
    n_trained = sum(p.numel() for p in r.parameters() if p.requires_grad)
    res = _base_result(args, w, world, value, elapsed, args.mlp_dtype + " MLP / f32 render")
    res.update({
        "data": "synthetic poses and decaying-noise target IRs; random-init AVRModel_complex (RAF widths)",
        "host_issue_ms_per_step": t_issue * 1e3 / args.steps,
        "config": {"workload": w.name, "mode": "ddp-train", "rays": R, "samples": S, "T": T,
                   "freq_bins": w.F, "poses_per_rank": B, "global_batch": B * world,
                   "model": "AVRModel_complex (6 hash grids, RAF MLP widths)",
                   "params": n_params, "grad_allreduce_bytes": 4 * n_params if world > 1 else 0,
                   "parallelism": f"dp{world} (DDP, RCCL bucketed gradient all-reduce)"},
        "roofline": adam_roofline(used, n_trained),
    })
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    what, n = resolve_world(args)
    if what == "launch":
        # start the ranks as children (never exec from this process)
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        return subprocess.call(launch_command(n, argv, free_port()), env=env)
    world = n
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local if world > 1 and not args.oversubscribe else 0)
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        if args.oversubscribe:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()

    from avr_amd.workloads import WORKLOADS

    w = WORKLOADS[args.workload]
    fn = {"pose": bench_pose, "ray-shard": bench_ray_shard, "ddp-train": bench_ddp_train}[args.mode]
    result = fn(args, w, world, rank, dev)
    if args.oversubscribe:
        result["oversubscribed"] = f"{world} ranks on cuda:0 over gloo (launcher rehearsal, not a scaling number)"
    attach_cpu_baseline(result, args, w, world, rank)
    if rank == 0 and world == 1 and args.mode == "pose" and w.name.startswith("c2_meshrir") \
            and not args.no_network:
        result["network_inference"] = network_inference(w, dev)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
