"""Repeated same-shape inference renders replayed from a HIP graph.

A config-2 pose is ~7 launches (sampling, weights, ray reduction, DFT,
finalize, irfft) behind Python and ctypes; issued eagerly, one pose's serial
latency carries that host time and the gaps between launches.
`GraphedRender` captures `AVRRender.render_ir` once per (batch, direction_tx,
device) with `torch.cuda.graph` and replays it:

    g = GraphedRender(renderer)
    spec, ir = g.render_ir(rays_o, position_tx)   # static output buffers

Per call, only the pose tensors and the azimuth jitter are refreshed: the
jitter is drawn from the CPU generator exactly as the eager path draws it
(renderer.py:149,153, same stream consumption), copied into a device buffer
that the captured sampling kernel reads at replay (`avr_sample_rays_dev`).
With the same seed the replay equals the eager render bit for bit
(tests/test_gpu_graph.py).

The network is captured too, so it must be graph-safe (no host syncs, same
tensors every call): the stub network of bench.py, and the package's own
models at inference.  The package's weight caches (bf16 casts, packed
head/sigma weights, bias columns) are bypassed while a graph is captured
(wcache.capturing), so every replay derives them from the master weights it
reads by pointer: an optimizer step (in place) between replays is seen, and
a parameter whose storage was replaced (load_state_dict with assign, .to())
starts a new capture (graphs are keyed on the parameters' data pointers).  The returned tensors are the graph's static outputs,
overwritten by the next replay of the same graph: clone them to keep them.
"""
from __future__ import annotations

from types import SimpleNamespace

import torch

from .renderer import draw_jitter


class GraphedRender:
    """HIP-graph replay of `AVRRender.render_ir` for fixed shapes."""

    def __init__(self, renderer, warmup: int = 2):
        self.renderer = renderer
        self.warmup = warmup
        self._graphs = {}

    def _capture(self, dev, rays_o, position_tx, direction_tx):
        r = self.renderer
        g = SimpleNamespace()
        g.ro = rays_o.detach().to(dev, torch.float32).clone()
        g.tx = position_tx.detach().to(dev, torch.float32).clone()
        g.dtx = None if direction_tx is None else direction_tx.detach().to(dev, torch.float32).clone()
        g.u = torch.zeros(int(r.n_azi), dtype=torch.float32, device=dev)
        # pinned staging ring for the per-call jitter: an async H2D copy,
        # each slot reused only after its previous copy completed
        g.ring = [torch.empty(int(r.n_azi), dtype=torch.float32, pin_memory=True) for _ in range(4)]
        g.ring_ev = [None] * 4
        g.slot = 0
        r._jitter_dev = g.u
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side), torch.no_grad():
                for _ in range(self.warmup):  # tables, caches, allocator pools
                    r.render_ir(g.ro, g.tx, g.dtx)
            torch.cuda.current_stream(dev).wait_stream(side)
            g.graph = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g.graph):
                g.out, g.ir = r.render_ir(g.ro, g.tx, g.dtx)
        finally:
            r._jitter_dev = None
        return g

    def render_ir(self, rays_o, position_tx, direction_tx=None):
        """(spectrum [B, F, 2], IR [B, 2(F-1)]) as `AVRRender.render_ir`,
        replayed; the tensors are the graph's static outputs."""
        r = self.renderer
        dev = r._device(rays_o)
        key = (int(position_tx.size(0)), direction_tx is None, dev,
               tuple(p.data_ptr() for p in r.parameters()))
        g = self._graphs.get(key)
        if g is None:
            g = self._graphs[key] = self._capture(dev, rays_o, position_tx, direction_tx)
        # one draw per render, as the eager path (CPU generator)
        k = g.slot
        g.slot = (k + 1) % len(g.ring)
        if g.ring_ev[k] is not None:
            g.ring_ev[k].synchronize()
        g.ring[k].copy_(draw_jitter(r.n_azi, r.n_ele))
        g.u.copy_(g.ring[k], non_blocking=True)
        ev = g.ring_ev[k] = g.ring_ev[k] or torch.cuda.Event()
        ev.record()
        if g.dtx is not None:
            torch._foreach_copy_([g.ro, g.tx, g.dtx], [rays_o, position_tx, direction_tx])
        else:
            torch._foreach_copy_([g.ro, g.tx], [rays_o, position_tx])
        g.graph.replay()
        return g.out, g.ir
