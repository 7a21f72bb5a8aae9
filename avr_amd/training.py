"""One training iteration of the reference loop (avr_runner.py:160-200) on
the MI355X path, and its checkpoint format (avr_runner.py:136-153, 105-130).

    step = TrainStep(renderer, cfg["train"], cfg["render"])
    losses = step(ori_sig, position_rx, position_tx)            # MeshRIR/Simu
    losses = step(ori_sig, position_rx, position_tx, direction_tx)  # RAF

Per call: render -> Criterion (HIP, all eight terms) -> sum -> backward ->
clip_grad_norm_(max_norm=1) + NaN/Inf zeroing (one HIP launch for all
gradients, `avr_scale_sanitize`) -> Adam -> CosineAnnealingLR, the order and
hyper-parameters of avr_runner.py:67-73, 181-200.  The reference's
`torch.isnan(energy_loss).item()` skip (avr_runner.py:183) is kept when
`nan_check=True` (the default, one host sync per step, as the reference).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .criterion import Criterion


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def clip_and_sanitize_(params, max_norm=1.0):
    """clip_grad_norm_(params, max_norm) followed by zeroing non-finite
    gradient entries (avr_runner.py:190-196), without a host sync.

    The total norm is torch's own (foreach per-tensor norms, then the norm of
    those); scaling and sanitising run as one HIP launch over every fp32
    gradient.  Returns the total norm (a device tensor), like clip_grad_norm_.
    """
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.zeros(())
    dev = grads[0].device
    if not grads[0].is_cuda:
        raise RuntimeError("clip_and_sanitize_ needs HIP tensors (no CPU fallback)")
    norms = torch._foreach_norm(grads, 2.0)
    total = torch.linalg.vector_norm(torch.stack([n.float() for n in norms]), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    fast = [g for g in grads if g.dtype == torch.float32 and g.is_contiguous() and g.device == dev]
    other = [g for g in grads if not (g.dtype == torch.float32 and g.is_contiguous() and g.device == dev)]
    if fast:
        ptrs = (ctypes.c_void_p * len(fast))(*[g.data_ptr() for g in fast])
        sizes = (ctypes.c_int64 * len(fast))(*[g.numel() for g in fast])
        with torch.cuda.device(dev):
            _lib.call("avr_scale_sanitize", len(fast), ptrs, sizes, coef.data_ptr(), _stream(dev))
    for g in other:  # non-fp32 / strided gradients: the same arithmetic with torch ops
        g.mul_(coef.to(g.device, g.dtype))
        g.nan_to_num_(nan=0.0, posinf=0.0, neginf=0.0)
    return total


class TrainStep:
    """avr_runner.py's optimiser, scheduler, criterion and inner-loop body."""

    def __init__(self, renderer, train_cfg, render_cfg, fused_adam=True, nan_check=True):
        self.renderer = renderer
        self.criterion = Criterion(train_cfg, render_cfg)
        self.optimizer = torch.optim.Adam(renderer.parameters(), lr=float(train_cfg['lr']),
                                          weight_decay=float(train_cfg.get('weight_decay', 0)),
                                          betas=(0.9, 0.999), fused=fused_adam)
        self.scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(
            optimizer=self.optimizer, T_max=float(train_cfg['T_max']),
            eta_min=float(train_cfg['eta_min']), last_epoch=-1)
        self.nan_check = nan_check
        self.current_iteration = 0

    def __call__(self, ori_sig, position_rx, position_tx, direction_tx=None, ch_idx=None):
        dev = next(self.renderer.parameters()).device
        args = [position_rx.to(dev), position_tx.to(dev)]
        if direction_tx is not None:
            args.append(direction_tx.to(dev))
        kw = {} if ch_idx is None or int(ch_idx.reshape(-1)[0]) == -1 else {"ch_idx": ch_idx.to(dev)}
        out = self.renderer(*args, **kw)
        losses = self.criterion(out, ori_sig.to(dev))
        if self.nan_check and torch.isnan(losses[4]).item():
            return None  # avr_runner.py:183-185: skip the step
        total = losses[0]
        for x in losses[1:8]:
            total = total + x
        self.optimizer.zero_grad(set_to_none=True)
        total.backward()
        clip_and_sanitize_(self.renderer.parameters(), max_norm=1)
        self.optimizer.step()
        self.scheduler.step()
        self.current_iteration += 1
        return total.detach(), [x.detach() for x in losses[:8]]

    # ------------------------------------------------------ checkpoints
    def save_checkpoint(self, path):
        """The reference's `.tar` layout (avr_runner.py:148-153)."""
        model = self.renderer.module if hasattr(self.renderer, "module") else self.renderer
        torch.save({
            'current_iteration': self.current_iteration,
            'audionerf_network_state_dict': model.state_dict(),
            'optimizer_state_dict': self.optimizer.state_dict(),
            'scheduler_state_dict': self.scheduler.state_dict(),
        }, path)
        return path

    def load_checkpoint(self, path):
        """avr_runner.py:105-130: restore weights, optimiser, scheduler, iteration."""
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        model = self.renderer.module if hasattr(self.renderer, "module") else self.renderer
        model.load_state_dict(ckpt['audionerf_network_state_dict'])
        self.optimizer.load_state_dict(ckpt['optimizer_state_dict'])
        self.scheduler.load_state_dict(ckpt['scheduler_state_dict'])
        self.current_iteration = int(ckpt['current_iteration'])
        return ckpt
