"""One training iteration of the reference loop (avr_runner.py:160-200) on
the MI355X path, and its checkpoint format (avr_runner.py:136-153, 105-130).

    step = TrainStep(renderer, cfg["train"], cfg["render"])
    losses = step(ori_sig, position_rx, position_tx)            # MeshRIR/Simu
    losses = step(ori_sig, position_rx, position_tx, direction_tx)  # RAF

Per call: render -> Criterion (HIP, all eight terms) -> sum -> backward ->
clip_grad_norm_(max_norm=1) + NaN/Inf zeroing + Adam (one HIP pass over
p, g, m, v: `avr_adam_step`) -> CosineAnnealingLR, the order and
hyper-parameters of avr_runner.py:67-73, 181-200.  The reference's
`torch.isnan(energy_loss).item()` skip (avr_runner.py:183) is kept when
`nan_check=True` (the default, one host sync per step, as the reference).
"""
from __future__ import annotations

import ctypes
import math

import torch
from torch.autograd.graph import increment_version

from . import _lib
from .criterion import Criterion


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _clip_coef(grads, max_norm):
    """clip_grad_norm_'s total norm and clamped coefficient, on the device."""
    norms = torch._foreach_norm(grads, 2.0)
    total = torch.linalg.vector_norm(torch.stack([n.float() for n in norms]), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return total, coef


def _native_clip_coef(grads, max_norm, dev):
    """_clip_coef's total norm and coefficient by `avr_grad_clip_coef`: one
    read of every gradient (torch's foreach norm + stack + norm + clamp take
    5-8 launches and ~2x the time), the same value within fp32 rounding."""
    n = len(grads)
    ptrs = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads])
    sizes = (ctypes.c_int64 * n)(*[g.numel() for g in grads])
    nb = ctypes.c_int64(0)
    _lib.call("avr_grad_clip_workspace", n, sizes, ctypes.byref(nb))
    work = torch.empty(max(1, nb.value // 4), dtype=torch.float32, device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    _lib.call("avr_grad_clip_coef", n, ptrs, sizes, float(max_norm), work.data_ptr(), nb.value,
              out.data_ptr(), out[1:].data_ptr(), _stream(dev))
    return out[0], out[1]


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
    total, coef = _clip_coef(grads, max_norm)
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


def _native_adam_ok(optimizer):
    for group in optimizer.param_groups:
        if group.get("amsgrad") or group.get("maximize") or group.get("differentiable"):
            return False
        for p in group["params"]:
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                return False
    return True


def clip_sanitize_adam_(optimizer, max_norm=1.0, events=None):
    """clip_and_sanitize_ + optimizer.step() of a torch.optim.Adam
    (avr_runner.py:190-200) as one HIP pass per parameter (`avr_adam_step`):
    p, g, m, v read once, p, m, v written once.

    The optimiser state stays in torch.optim.Adam's own (non-fused) layout --
    `step` a CPU float tensor, `exp_avg`, `exp_avg_sq` -- so state_dict(),
    load_state_dict(), checkpoints and the LR scheduler are unchanged.  The
    clipped, sanitised gradient is consumed inside the kernel and not written
    back to p.grad (the loop zeroes it before the next backward).  Returns the
    total norm (a device tensor).  `events`: an optional (begin, end) pair of
    torch.cuda.Event recorded around the Adam launches (bench.py's roofline).
    """
    params = [p for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
    if not params:
        return torch.zeros(())
    dev = params[0].device
    grads = [p.grad for p in params]
    if all(g.dtype == torch.float32 and g.is_contiguous() and g.device == dev for g in grads):
        total, coef = _native_clip_coef(grads, max_norm, dev)
    else:
        total, coef = _clip_coef(grads, max_norm)
    st_ = _stream(dev)
    if events is not None and events[0] is not None:
        events[0].record()
    for group in optimizer.param_groups:
        b1, b2 = group["betas"]
        lr = float(group["lr"])
        ps, gs, ms, vs, ns, ss, bs = [], [], [], [], [], [], []
        for p in group["params"]:
            if p.grad is None:
                continue
            g = p.grad
            if not (g.dtype == torch.float32 and g.is_contiguous()):
                raise RuntimeError("clip_sanitize_adam_: gradients must be contiguous fp32")
            st = optimizer.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if st["step"].is_cuda:  # state loaded from a fused/capturable optimiser
                st["step"] = st["step"].cpu()
            st["step"] += 1
            step = float(st["step"])
            ps.append(p.data_ptr())
            gs.append(g.data_ptr())
            ms.append(st["exp_avg"].data_ptr())
            vs.append(st["exp_avg_sq"].data_ptr())
            ns.append(p.numel())
            ss.append(lr / (1.0 - b1 ** step))
            bs.append(math.sqrt(1.0 - b2 ** step))
        if not ps:
            continue
        # the kernel writes through raw pointers: bump the version counters as
        # torch's in-place update would, so version-keyed caches (wcache, the
        # packed sigma / head weights) see the new values
        increment_version([p for p in group["params"] if p.grad is not None])
        n = len(ps)
        arr = lambda t, xs: (t * n)(*xs)  # noqa: E731
        with torch.cuda.device(dev):
            _lib.call("avr_adam_step", n, arr(ctypes.c_void_p, ps), arr(ctypes.c_void_p, gs),
                      arr(ctypes.c_void_p, ms), arr(ctypes.c_void_p, vs), arr(ctypes.c_int64, ns),
                      arr(ctypes.c_float, ss), arr(ctypes.c_float, bs), float(b1), float(b2),
                      float(group["eps"]), float(group["weight_decay"]), coef.data_ptr(), st_)
    if events is not None and events[1] is not None:
        events[1].record()
    return total


class TrainStep:
    """avr_runner.py's optimiser, scheduler, criterion and inner-loop body."""

    def __init__(self, renderer, train_cfg, render_cfg, fused_adam=True, nan_check=True, native_adam=True):
        self.renderer = renderer
        self.criterion = Criterion(train_cfg, render_cfg)
        # native_adam: clip + sanitize + Adam in one HIP pass (clip_sanitize_adam_);
        # the Adam object then only holds state (reference's non-fused layout)
        self.optimizer = torch.optim.Adam(renderer.parameters(), lr=float(train_cfg['lr']),
                                          weight_decay=float(train_cfg.get('weight_decay', 0)),
                                          betas=(0.9, 0.999), fused=fused_adam and not native_adam)
        self.native_adam = native_adam and _native_adam_ok(self.optimizer)
        self.scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(
            optimizer=self.optimizer, T_max=float(train_cfg['T_max']),
            eta_min=float(train_cfg['eta_min']), last_epoch=-1)
        self.nan_check = nan_check
        self.current_iteration = 0
        # instrumentation: a callable returning the (begin, end) events to
        # record around this step's Adam launches, or None (bench.py)
        self.adam_events = None

    def __call__(self, ori_sig, position_rx, position_tx, direction_tx=None, ch_idx=None):
        dev = next(self.renderer.parameters()).device
        args = [position_rx.to(dev), position_tx.to(dev)]
        if direction_tx is not None:
            args.append(direction_tx.to(dev))
        kw = {} if ch_idx is None or int(ch_idx.reshape(-1)[0]) == -1 else {"ch_idx": ch_idx.to(dev)}
        out = self.renderer(*args, **kw)
        # total_loss = spec + ... + das_ce (avr_runner.py:187), summed in the
        # criterion's reduce kernel
        losses, total = self.criterion.forward_total(out, ori_sig.to(dev))
        if self.nan_check and torch.isnan(losses[4]).item():
            return None  # avr_runner.py:183-185: skip the step
        self.optimizer.zero_grad(set_to_none=True)
        total.backward()
        if self.native_adam:
            clip_sanitize_adam_(self.optimizer, max_norm=1,
                                events=self.adam_events() if self.adam_events is not None else None)
            # the Adam update ran natively: tell the LR scheduler that this
            # step's optimizer.step() happened (its order check reads the flag)
            self.optimizer._opt_called = True
        else:
            clip_and_sanitize_(self.renderer.parameters(), max_norm=1)
            self.optimizer.step()
        self.scheduler.step()
        self.current_iteration += 1
        return total.detach(), [x.detach() for x in losses[:8]]

    # ------------------------------------------------------ checkpoints
    def save_checkpoint(self, path, reference_layout=False):
        """The reference's `.tar` layout (avr_runner.py:148-153).  With
        `reference_layout` the networks are written as tcnn's flat `params`
        (avr_amd.tcnn_compat) and the Adam state is converted to the same
        parameters (one flat exp_avg / exp_avg_sq per tcnn module, in the
        reference's module order), the form the reference's runner loads:
        `load_state_dict` of the weights, then `optimizer.load_state_dict`
        (avr_runner.py:116-124)."""
        from .tcnn_compat import optimizer_state_to_reference, to_reference

        model = self.renderer.module if hasattr(self.renderer, "module") else self.renderer
        opt = self.optimizer.state_dict()
        torch.save({
            'current_iteration': self.current_iteration,
            'audionerf_network_state_dict': to_reference(model) if reference_layout else model.state_dict(),
            'optimizer_state_dict': optimizer_state_to_reference(model, opt) if reference_layout else opt,
            'scheduler_state_dict': self.scheduler.state_dict(),
        }, path)
        return path

    def load_checkpoint(self, path):
        """avr_runner.py:105-130: restore weights, optimiser, scheduler, iteration.

        A checkpoint written by the reference (tcnn networks: one flat
        `params` per network) is recognised and converted
        (avr_amd.tcnn_compat.from_reference), its Adam state too
        (optimizer_state_from_reference).  When that state does not fit this
        model's parameters (another parameter count or size), the optimiser
        starts fresh and a warning says so."""
        import warnings

        from .tcnn_compat import from_reference, is_reference_layout, optimizer_state_from_reference

        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        model = self.renderer.module if hasattr(self.renderer, "module") else self.renderer
        sd = ckpt['audionerf_network_state_dict']
        opt_sd = ckpt['optimizer_state_dict']
        if is_reference_layout(model, sd):
            from_reference(model, sd)
            try:
                opt_sd = optimizer_state_from_reference(model, opt_sd,
                                                        self.optimizer.state_dict()["param_groups"])
            except ValueError as e:
                warnings.warn(f"reference checkpoint: {e}; optimizer state not restored", RuntimeWarning)
                opt_sd = None
        else:
            model.load_state_dict(sd)
        if opt_sd is not None:
            self.optimizer.load_state_dict(opt_sd)
        self.scheduler.load_state_dict(ckpt['scheduler_state_dict'])
        self.current_iteration = int(ckpt['current_iteration'])
        return ckpt
