"""Repeated same-shape inference renders replayed from a HIP graph.

A config-2 pose is 6 launches (sampling, weights, ray reduction, DFT,
finalize, irfft) behind Python and ctypes; issued eagerly, one pose's serial
latency carries that host time and the gaps between launches.
`GraphedRender` captures `AVRRender.render_ir` per (batch, direction_tx,
device, parameters) with `torch.cuda.graph` and replays it:

    g = GraphedRender(renderer)
    spec, ir = g.render_ir(rays_o, position_tx)   # static output buffers

Per call, only the pose and the azimuth jitter are refreshed, and no
host-to-device copy precedes the replay.  The jitter is drawn from the CPU
generator exactly as the eager path draws it (renderer.py:149,153, same
stream consumption) straight into a pinned, device-mapped host buffer
(`avr_pinned_alloc`) that the captured sampling kernel reads at replay.
Poses given as host tensors (as a data loader yields them,
avr_runner.py:168) are written into the same buffer, ahead of the jitter,
and the sampling kernel publishes them to device memory for the later
kernels (`avr_sample_rays_staged`); poses already on the device are copied
into the graph's static pose tensors by one launch before the replay
(`avr_sample_rays_dev` then reads only the jitter from the host buffer).
Because a graph's kernel arguments are fixed, each key holds a small ring
of captured instances, each with its own host buffer and static tensors; an
instance is reused only after its previous replay has finished (an event
per instance), so pipelined replays never see a buffer rewritten under
them.  With the same seed the replay equals the eager render bit for bit
(tests/test_gpu_graph.py).

The network is captured too, so it must be graph-safe (no host syncs, same
tensors every call): the stub network of bench.py, and the package's own
models at inference.  The package's weight caches (bf16 casts, packed
head/sigma weights, bias columns) are bypassed while a graph is captured
(wcache.capturing), so every replay derives them from the master weights it
reads by pointer: an optimizer step (in place) between replays is seen, and
a parameter whose storage was replaced (load_state_dict with assign, .to())
starts a new capture (graphs are keyed on the parameters' data pointers).
The returned tensors are the instance's static outputs, overwritten when
the ring comes back to it (`ring` calls later): clone them to keep them.
"""
from __future__ import annotations

import ctypes
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib


class PinnedHostBuffer:
    """fp32 host memory the GPU reads directly (avr_pinned_alloc): `.host`
    is a CPU tensor view of it, `.dev_ptr` the address kernels use."""

    def __init__(self, n: int):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("avr_pinned_alloc", 4 * n, ctypes.byref(h), ctypes.byref(d))
        self._h = h.value
        self.dev_ptr = d.value
        arr = np.ctypeslib.as_array((ctypes.c_float * n).from_address(self._h))
        self.host = torch.from_numpy(arr)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self.host = None
            try:
                _lib.load().avr_pinned_free(h)
            except Exception:  # interpreter shutdown: the process frees it
                pass


class GraphedRender:
    """HIP-graph replay of `AVRRender.render_ir` for fixed shapes."""

    def __init__(self, renderer, warmup: int = 2, ring: int = 3):
        self.renderer = renderer
        self.warmup = warmup
        self.ring = max(1, int(ring))
        self._graphs = {}  # key -> [instances], next index
        self._dev_cache = {}  # current device index -> torch.device

    def _capture(self, dev, rays_o, position_tx, direction_tx, warmup):
        r = self.renderer
        B = int(position_tx.size(0))
        n_azi, n_ele = int(r.n_azi), int(r.n_ele)
        g = SimpleNamespace(host_pose=not rays_o.is_cuda, has_dtx=direction_tx is not None, B=B)
        # [rays_o | pos_tx | dir_tx | u_azi | elevation draws (consumed, unused)]
        g.buf = PinnedHostBuffer(9 * B + n_azi + n_ele)
        g.buf.host.zero_()
        g.pose_h = g.buf.host[:9 * B]
        g.jit_h = g.buf.host[9 * B:]
        g.done = None
        if g.host_pose:
            g.pose_dev = torch.zeros(9 * B, dtype=torch.float32, device=dev)
            g.ro, g.tx = g.pose_dev[:3 * B].view(B, 3), g.pose_dev[3 * B:6 * B].view(B, 3)
            g.dtx = g.pose_dev[6 * B:].view(B, 3) if g.has_dtx else None
            r._staged = (g.buf.dev_ptr, g.pose_dev)
        else:
            g.ro = rays_o.detach().to(dev, torch.float32).clone()
            g.tx = position_tx.detach().to(dev, torch.float32).clone()
            g.dtx = None if direction_tx is None else direction_tx.detach().to(dev, torch.float32).clone()
            r._jitter_dev = g.buf.dev_ptr + 4 * 9 * B
        try:
            if warmup:
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side), torch.no_grad():
                    for _ in range(warmup):  # tables, caches, allocator pools
                        r.render_ir(g.ro, g.tx, g.dtx)
                torch.cuda.current_stream(dev).wait_stream(side)
                side.synchronize()
            g.graph = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g.graph):
                g.out, g.ir = r.render_ir(g.ro, g.tx, g.dtx)
            # networks that declare `draws_no_device_rng` (ours; no dropout)
            # are replayed by avr_graph_launch: the render itself draws on the
            # CPU, so torch's replay prologue (device-RNG seed/offset refresh)
            # has nothing to do.  Any other network keeps CUDAGraph.replay.
            g.exec = (int(g.graph.raw_cuda_graph_exec())
                      if getattr(r.network_fn, "draws_no_device_rng", False) else None)
            g.pose_np = g.pose_h.numpy()
            g.jit_n = n_azi + n_ele
        finally:
            r._jitter_dev = None
            r._staged = None
        return g

    def render_ir(self, rays_o, position_tx, direction_tx=None):
        """(spectrum [B, F, 2], IR [B, 2(F-1)]) as `AVRRender.render_ir`,
        replayed; the tensors are the instance's static outputs.  Host
        (CPU) pose tensors take the staged path, device ones one copy."""
        r = self.renderer
        # the device without r._device's availability check and torch.device
        # construction on every call (~1 us of the serial pose); a host pose
        # renders on the current device, as the eager path does
        dev = rays_o.device if rays_o.is_cuda else self._dev_cache.get(torch.cuda.current_device())
        if dev is None:
            dev = self._dev_cache.setdefault(torch.cuda.current_device(), r._device(rays_o))
        key = (int(position_tx.size(0)), direction_tx is None, rays_o.is_cuda, dev,
               tuple(p.data_ptr() for p in r.parameters()))
        slot = self._graphs.get(key)
        if slot is None:
            slot = self._graphs[key] = [[], 0]
        insts, k = slot
        if k >= len(insts):
            insts.append(self._capture(dev, rays_o, position_tx, direction_tx,
                                       self.warmup if not insts else 0))
        g = insts[k]
        slot[1] = (k + 1) % self.ring
        if g.done is not None and not g.done.query():
            g.done.synchronize()  # its previous replay has read the buffer
        # the eager path's two CPU-generator draws (renderer.draw_jitter) in
        # one call (the generator fills them in order: tests/test_graph_cpu.py),
        # straight into the buffer the captured kernel reads
        torch.rand(g.jit_n, out=g.jit_h)
        B = g.B
        if g.host_pose:
            poses = (rays_o, position_tx, direction_tx) if g.has_dtx else (rays_o, position_tx)
            nb = 12 * B
            for k, t in enumerate(poses):
                if (t.dtype is torch.float32 and t.device.type == "cpu" and t.numel() == 3 * B
                        and t.is_contiguous()):
                    # one memmove into the pinned buffer: no dispatcher call
                    ctypes.memmove(g.buf._h + k * nb, t.data_ptr(), nb)
                else:
                    # another dtype or layout, or a device tensor beside host
                    # rays_o (the eager path accepts mixed devices)
                    v = t.detach().reshape(-1).float().cpu()
                    if v.numel() != 3 * B:
                        raise ValueError(f"GraphedRender: pose tensor {tuple(t.shape)} is not [{B}, 3]")
                    g.pose_np[3 * B * k:3 * B * (k + 1)] = v.numpy()
        elif g.dtx is not None:
            torch._foreach_copy_([g.ro, g.tx, g.dtx], [rays_o, position_tx, direction_tx])
        else:
            torch._foreach_copy_([g.ro, g.tx], [rays_o, position_tx])
        if g.exec is not None:
            lib = _lib.load()
            if lib.avr_graph_launch(g.exec, torch._C._cuda_getCurrentRawStream(dev.index)) != 0:
                raise RuntimeError(f"avr_graph_launch failed: {lib.avr_last_error().decode(errors='replace')}")
        else:
            g.graph.replay()
        g.done = g.done or torch.cuda.Event()
        g.done.record()
        return g.out, g.ir
