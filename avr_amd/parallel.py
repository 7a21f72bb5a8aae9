"""Multi-GPU decomposition of the render path.

One process per GPU over `torch.distributed` (backend "nccl" = RCCL on ROCm,
xGMI inside a node).  Two shardings, both exact because the reference's
output is a plain sum over rays (renderer.py:118) and poses are
independent:

* poses  — `shard_range(B, rank, world)`: each rank renders its own poses,
  no data-path collective (inference of batches; training under DDP, whose
  bucketed gradient all-reduce replaces avr_runner_ddp.py:98).
* rays   — `RayShardedRender`: a single pose's rays are split into
  contiguous ranges; every rank renders a partial spectrum [B, F, 2] and one
  all-reduce (F*8 bytes per pose: 4 KiB at config 2) sums them.  The azimuth
  jitter is drawn on every rank (keeping each rank's CPU generator in the
  same state as the reference's) and rank 0's draw is broadcast, so all
  shards see one sphere.  Over RCCL the broadcast stays on the device and the
  sampling kernel reads the jitter there (no host synchronisation per pose).

  Training through a ray-sharded render: the loss on the all-reduced
  spectrum is replicated, so each rank's parameter gradient covers only its
  own rays and the true gradient is their SUM.  Call
  `allreduce_grads_sum(module.parameters())` after backward (do not wrap the
  module in DDP, which would average).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from .renderer import draw_jitter


def shard_range(n: int, rank: int, world: int):
    """Contiguous balanced split of range(n): the first n % world ranks get one more."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class _AllReduceSum(torch.autograd.Function):
    """Sum over ranks in forward; identity in backward (the loss on the
    all-reduced output is replicated, so each rank's partial receives the
    same upstream gradient)."""

    @staticmethod
    def forward(ctx, x, group):
        y = x.clone()
        dist.all_reduce(y, op=dist.ReduceOp.SUM, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


def allreduce_spectrum(partial: torch.Tensor, group=None) -> torch.Tensor:
    return _AllReduceSum.apply(partial, group)


def broadcast_jitter(u_azi: torch.Tensor, group=None, device=None, keep_on_device=False) -> torch.Tensor:
    """Rank 0's azimuth draw to every rank (n_azi floats).

    With `keep_on_device` (RCCL) the result stays a device tensor, which
    `AVRRender.sample` reads in its sampling kernel without a host copy."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return u_azi
    backend = dist.get_backend(group)
    t = u_azi.to(device) if (backend == "nccl" and device is not None) else u_azi.clone()
    dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return t if (keep_on_device and t.is_cuda) else t.cpu()


def allreduce_grads_sum(params, group=None):
    """SUM-all-reduce of parameter gradients after a ray-sharded backward
    (each rank's gradient covers its own rays; the full-pose gradient is
    their sum).  One flat buffer per dtype/device, one collective each."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    buckets = {}
    for p in params:
        if p.grad is not None:
            buckets.setdefault((p.grad.device, p.grad.dtype), []).append(p.grad)
    for grads in buckets.values():
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n


class RayShardedRender(nn.Module):
    """Render one batch of poses with its rays split over the ranks of `group`.

    Wraps an `avr_amd.AVRRender`; `network_fn` is called only on this rank's
    rays.  Returns the full [B, F, 2] spectrum on every rank.

    `shard=(rank, world)` (one process, no collective): render only that
    shard's rays and return its partial spectrum -- one rank's work of a
    world-rank job, measured on a single GPU (bench.py --shard-of).
    """

    def __init__(self, renderer, group=None, shard=None):
        super().__init__()
        self.renderer = renderer
        self.group = group
        self.shard = shard

    def forward(self, rays_o, position_tx, direction_tx=None, ch_idx=None):
        r = self.renderer
        if self.shard is not None:
            rank, world = self.shard
        else:
            world = dist.get_world_size(self.group) if dist.is_initialized() else 1
            rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        R = int(r.n_azi) * int(r.n_ele) + 2
        r.ray_range = shard_range(R, rank, world)
        try:
            u = broadcast_jitter(draw_jitter(r.n_azi, r.n_ele), self.group, rays_o.device,
                                 keep_on_device=rays_o.is_cuda)
            # the renderer's own path on this rank's rays: the network is told
            # the shard's ray layout (per-ray / per-pose encodings once) and a
            # fused-head network renders through FusedHeadCore (the exact
            # 16-bit head), exactly as an unsharded render
            partial = r._render(rays_o, position_tx, direction_tx, ch_idx, None, u_azi=u)
        finally:
            r.ray_range = None
        if world == 1 or self.shard is not None:
            return partial
        return allreduce_spectrum(partial, self.group)


def ddp(module: nn.Module, device, bucket_cap_mb: int = 64, **kw):
    """DistributedDataParallel over RCCL for training (config 4).

    Gradients are all-reduced in buckets during backward; 64 MiB buckets keep
    the ~236 MB of RAF hash-grid + MLP gradients to a handful of ring
    collectives, each large enough to saturate the per-link xGMI bandwidth.
    """
    from torch.nn.parallel import DistributedDataParallel as DDP

    return DDP(module, device_ids=[device.index] if device is not None and device.type == "cuda" else None,
               bucket_cap_mb=bucket_cap_mb, **kw)
