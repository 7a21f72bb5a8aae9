"""CPU, world_size 2 over gloo: the multi-GPU decomposition logic.

Ray sharding is exact because the reference sums the per-ray spectra
(renderer.py:118): rendering each rank's contiguous ray range and
all-reducing must reproduce the single-process result.  Checked here with
the CPU oracle standing in for the per-rank render (rays outside the shard
contribute zero signal)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from avr_amd.parallel import allreduce_grads_sum, allreduce_spectrum, broadcast_jitter, shard_range
from avr_amd.workloads import WORKLOADS, make_inputs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import avr_oracle as orc

        res = {}
        # 1. jitter broadcast: ranks start from different generator states
        torch.manual_seed(100 + rank)
        u = broadcast_jitter(torch.rand(7))
        torch.manual_seed(100)
        res["jitter_ok"] = bool(torch.equal(u, torch.rand(7)))

        # 2. ray-sharded render == full render
        w = WORKLOADS["c1_meshrir_plumbing"]
        inp = make_inputs(w, 1)
        R, S, T = w.n_rays, w.n_samples, w.T
        r0, r1 = shard_range(R, rank, world)
        sig = inp["signal"].reshape(1, R, S, T).copy()
        sig[:, :r0] = 0
        sig[:, r1:] = 0
        cfg = orc.RenderConfig.from_kwargs(**w.render)
        torch.manual_seed(1)
        part = orc.render_spectrum(cfg, orc.StubNetwork(torch.from_numpy(inp["attn"]),
                                                        torch.from_numpy(sig.reshape(inp["signal"].shape))),
                                   torch.from_numpy(inp["rays_o"]), torch.from_numpy(inp["position_tx"]))
        part.requires_grad_(True)
        full = allreduce_spectrum(part)
        torch.manual_seed(1)
        ref = orc.render_spectrum(cfg, orc.StubNetwork(torch.from_numpy(inp["attn"]),
                                                       torch.from_numpy(inp["signal"])),
                                  torch.from_numpy(inp["rays_o"]), torch.from_numpy(inp["position_tx"]))
        res["rel"] = float((full.detach() - ref).norm() / ref.norm())
        g = torch.randn(full.shape, generator=torch.Generator().manual_seed(3))
        (full * g).sum().backward()
        res["grad_ok"] = bool(torch.equal(part.grad, g))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    for n in (1, 7, 32, 1024, 4096):
        for world in (1, 2, 3, 8):
            if world > n:
                continue
            ranges = [shard_range(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_ray_sharded_render_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in out.items():
        assert res["jitter_ok"], rank
        assert res["rel"] < 1e-6, res
        assert res["grad_ok"], rank


def _ddp_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from avr_amd.parallel import ddp, shard_range

        torch.manual_seed(0)
        net = torch.nn.Linear(8, 4, bias=False)
        model = ddp(net, None)
        # each rank takes its own pose shard of a batch of 6 (DistributedSampler-like)
        x = torch.randn(6, 8, generator=torch.Generator().manual_seed(1))
        a, b = shard_range(6, rank, world)
        model(x[a:b]).pow(2).sum().backward()
        q.put((rank, net.weight.grad.tolist()))  # plain data: the sender exits right after
    finally:
        dist.destroy_process_group()


def test_ddp_helper_allreduces_pose_shard_grads_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    ref = torch.nn.Linear(8, 4, bias=False)
    x = torch.randn(6, 8, generator=torch.Generator().manual_seed(1))
    ref(x).pow(2).sum().backward()
    # DDP averages over ranks: mean of the two shard gradients
    for g in out.values():
        torch.testing.assert_close(torch.tensor(g), ref.weight.grad / 2, rtol=1e-5, atol=1e-6)


def _ray_grad_worker(rank, world, port, q):
    """Ray-sharded TRAINING: parameter gradients summed over ranks equal the
    unsharded render's gradient (the loss on the all-reduced spectrum is
    replicated; each rank's backward covers only its own rays)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import avr_oracle as orc

        w = WORKLOADS["c1_meshrir_plumbing"]
        inp = make_inputs(w, 1)
        R, S, T = w.n_rays, w.n_samples, w.T
        cfg = orc.RenderConfig.from_kwargs(**w.render)
        base = torch.from_numpy(inp["signal"]).reshape(1, R, S, T)
        attn0 = torch.from_numpy(inp["attn"])
        g = torch.randn(1, T // 2 + 1, 2, generator=torch.Generator().manual_seed(5))

        def loss_and_grads(mask_rays):
            scale = torch.nn.Parameter(torch.linspace(0.5, 1.5, T))
            gain = torch.nn.Parameter(torch.tensor(1.25))
            sig = base * scale * mask_rays.view(1, R, 1, 1)
            torch.manual_seed(1)
            out = orc.render_spectrum(cfg, orc.StubNetwork(attn0 * gain, sig.reshape(1, R * S, T)),
                                      torch.from_numpy(inp["rays_o"]), torch.from_numpy(inp["position_tx"]))
            return out, (scale, gain)

        r0, r1 = shard_range(R, rank, world)
        m = torch.zeros(R)
        m[r0:r1] = 1
        part, params = loss_and_grads(m)
        full = allreduce_spectrum(part)
        (full * g).sum().backward()
        allreduce_grads_sum(params)
        ref, rparams = loss_and_grads(torch.ones(R))
        (ref * g).sum().backward()
        q.put((rank, [float((p.grad - rp.grad).abs().max() / rp.grad.abs().max().clamp(min=1e-30))
                      for p, rp in zip(params, rparams)]))
    finally:
        dist.destroy_process_group()


def test_ray_sharded_param_grads_sum_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ray_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, errs in out.items():
        assert max(errs) < 1e-5, (rank, errs)
