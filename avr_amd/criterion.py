"""Training criterion on the GPU: drop-in for `utils/criterion.py:Criterion`.

`Criterion(cfg, cfg_render)` reads the same `train:` keys
(criterion.py:11-21) and `forward(pred_sig, ori_sig)` returns the same
10-tuple (criterion.py:124-126):

    (spec_loss, amplitude_loss, angle_loss, time_loss, energy_loss,
     multi_stft_loss, das_reg_loss, das_ce_loss, ori_time, pred_time)

`pred_sig`, `ori_sig` are complex [B, F] (the training loop builds
`pred_sig = out[..., 0] + 1j * out[..., 1]`, avr_runner.py:178).  All terms
run in the HIP kernels of `csrc/criterion.hip` (forward: 3 launches, backward:
3 launches) through the C-ABI `avr_criterion_*`; gradients flow back to
`pred_sig` through a `torch.autograd.Function`.  The multi-resolution STFT
term restates `auraloss.freq.MultiResolutionSTFTLoss` (auraloss 0.4.0, absent
here) — see oracle/criterion_oracle.py for the statement of both.

There is no CPU path: a CPU tensor raises.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .renderer import _ir_twiddle

LOSS_KEYS = ("spec_loss_weight", "amplitude_loss_weight", "angle_loss_weight",
             "time_loss_weight", "energy_loss_weight", "multistft_loss_weight")
# criterion.py:33 (window lengths of the MR-STFT resolutions) and :74 (n_fft)
_MR_WIN = (300, 150, 75, 30)
_ENERGY_NFFT = 256

_TABLES: dict = {}
_TABLE_LOCK = threading.Lock()


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _window_table(dev):
    """hann windows exactly as auraloss builds them (torch.hann_window on the
    CPU, moved to the device) followed by the energy STFT's rectangular window."""
    key = ("win", dev.index)
    t = _TABLES.get(key)
    if t is None:
        with _TABLE_LOCK:
            t = _TABLES.get(key)
            if t is None:
                parts = [torch.hann_window(w) for w in _MR_WIN] + [torch.ones(_ENERGY_NFFT)]
                host = torch.cat(parts).float()
                assert host.numel() == _lib.load().avr_criterion_window_len()
                t = host.to(dev)
                _TABLES[key] = t
    return t


class _CriterionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, ori, weights, with_total=False):
        # pred, ori: [B, F, 2] fp32 contiguous device tensors; with_total: a
        # last output, the eight losses' sum (avr_criterion_fwd2)
        B, F = pred.size(0), pred.size(1)
        n = 2 * (F - 1)
        dev = pred.device
        win = _window_table(dev)
        tw512 = _ir_twiddle(512, dev)
        irtw = _ir_twiddle(n, dev)
        nbytes = _ws_bytes(B, F)
        ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        pred_time = torch.empty(B, n, dtype=torch.float32, device=dev)
        ori_time = torch.empty(B, n, dtype=torch.float32, device=dev)
        losses = torch.empty(9 if with_total else 8, dtype=torch.float32, device=dev)
        wts = (ctypes.c_float * 6)(*weights)
        with torch.cuda.device(dev):
            _lib.call("avr_criterion_fwd2", B, F, wts, _ptr(pred), _ptr(ori), _ptr(win),
                      _ptr(tw512), _ptr(irtw), _ptr(pred_time), _ptr(ori_time), _ptr(losses),
                      _ptr(losses[8:]) if with_total else None, _ptr(ws), nbytes, _stream(dev))
        ctx.save_for_backward(pred, ori, pred_time, ori_time, ws)
        ctx.weights = weights
        ctx.set_materialize_grads(False)
        ls = losses.unbind(0)
        ctx.mark_non_differentiable(ls[6], ls[7], ori_time)
        if with_total:
            return (*ls[:8], ori_time, pred_time, ls[8])
        return (*ls, ori_time, pred_time)

    @staticmethod
    def backward(ctx, *grads):
        pred, ori, pred_time, ori_time, ws = ctx.saved_tensors
        B, F = pred.size(0), pred.size(1)
        dev = pred.device
        gl = grads[:6]
        g_pt = grads[9]
        g_tot = grads[10] if len(grads) > 10 else None
        if all(g is None for g in gl) and g_pt is None and g_tot is None:
            return None, None, None, None
        if all(g is None for g in gl) and g_tot is not None:
            # d total / d loss_i = 1: each of the six losses gets total's grad
            g_losses = g_tot.reshape(1).float().expand(6).contiguous()
        else:
            zero = None
            parts = []
            for g in gl:
                if g is None:
                    if zero is None:
                        zero = torch.zeros((), dtype=torch.float32, device=dev)
                    g = zero
                parts.append(g.reshape(()).float())
            g_losses = torch.stack(parts)
            if g_tot is not None:
                g_losses = g_losses + g_tot.reshape(()).float()
        if g_pt is not None:
            g_pt = g_pt.float().contiguous()
        grad_pred = torch.empty_like(pred)
        n = 2 * (F - 1)
        wts = (ctypes.c_float * 6)(*ctx.weights)
        with torch.cuda.device(dev):
            _lib.call("avr_criterion_bwd", B, F, wts, _ptr(pred), _ptr(ori), _ptr(pred_time),
                      _ptr(ori_time), _ptr(g_losses), _ptr(g_pt), _ptr(_window_table(dev)),
                      _ptr(_ir_twiddle(512, dev)), _ptr(_ir_twiddle(n, dev)), _ptr(ws),
                      ws.numel() * 4, _ptr(grad_pred), _stream(dev))
        return grad_pred, None, None, None


_WS: dict = {}


def _ws_bytes(B, F):
    key = (B, F)
    v = _WS.get(key)
    if v is None:
        out = ctypes.c_int64(0)
        _lib.call("avr_criterion_workspace", B, F, ctypes.byref(out))
        v = int(out.value)
        _WS[key] = v
    return v


def _as_spectrum(sig, name):
    """complex [B, F] (or real [B, F, 2]) -> fp32 [B, F, 2] contiguous view."""
    if sig.is_complex():
        sig = torch.view_as_real(sig.to(torch.complex64))
    if sig.dim() != 3 or sig.size(-1) != 2:
        raise ValueError(f"{name}: expected complex [B, F] or real [B, F, 2], got {tuple(sig.shape)}")
    return sig.float().contiguous()


class Criterion(nn.Module):
    """utils/criterion.py:7-126 on the GPU (HIP kernels, no CPU fallback)."""

    def __init__(self, cfg, cfg_render):
        super().__init__()
        self.spec_loss_weight = cfg['spec_loss_weight']
        self.amplitude_loss_weight = cfg['amplitude_loss_weight']
        self.angle_loss_weight = cfg['angle_loss_weight']
        self.time_loss_weight = cfg['time_loss_weight']
        self.energy_loss_weight = cfg['energy_loss_weight']
        self.multi_stft_weight = cfg['multistft_loss_weight']
        self.das_reg_loss_weight = cfg.get('das_reg_loss_weight', 0.0)
        self.das_ce_loss_weight = cfg.get('das_ce_loss_weight', 0.0)
        self.beta = cfg.get('beta', 100.0)
        self.fs = cfg_render['fs']
        self.sound_speed = cfg_render['speed']
        self.K = 360

    def _weights(self):
        return tuple(float(np.float32(w)) for w in (
            self.spec_loss_weight, self.amplitude_loss_weight, self.angle_loss_weight,
            self.time_loss_weight, self.energy_loss_weight, self.multi_stft_weight))

    def forward(self, pred_sig, ori_sig):
        if not pred_sig.is_cuda:
            raise RuntimeError("avr_amd.Criterion needs HIP tensors (no CPU fallback)")
        pred = _as_spectrum(pred_sig, "pred_sig")
        ori = _as_spectrum(ori_sig, "ori_sig").detach()
        if pred.shape != ori.shape:
            raise ValueError(f"pred_sig {tuple(pred.shape)} and ori_sig {tuple(ori.shape)} differ")
        out = _CriterionFn.apply(pred, ori, self._weights())
        return self._with_das(out[:10])

    def forward_total(self, pred_sig, ori_sig):
        """(forward's ten outputs, total): total = the eight losses added left
        to right (avr_runner.py:187), from the criterion's own kernel when the
        DAS terms are off (seven torch adds otherwise)."""
        if self.das_reg_loss_weight > 0 or self.das_ce_loss_weight > 0:
            out = self.forward(pred_sig, ori_sig)
            total = out[0]
            for x in out[1:8]:
                total = total + x
            return out, total
        if not pred_sig.is_cuda:
            raise RuntimeError("avr_amd.Criterion needs HIP tensors (no CPU fallback)")
        pred = _as_spectrum(pred_sig, "pred_sig")
        ori = _as_spectrum(ori_sig, "ori_sig").detach()
        if pred.shape != ori.shape:
            raise ValueError(f"pred_sig {tuple(pred.shape)} and ori_sig {tuple(ori.shape)} differ")
        out = _CriterionFn.apply(pred, ori, self._weights(), True)
        return tuple(out[:10]), out[10]

    def _with_das(self, out):
        spec, amp, angle, time, energy, mr, das_reg, das_ce, ori_time, pred_time = out
        if self.das_reg_loss_weight > 0 or self.das_ce_loss_weight > 0:
            from .das import das_losses
            das_reg, das_ce = das_losses(pred_time, ori_time, self.fs, self.sound_speed,
                                         self.das_reg_loss_weight, self.das_ce_loss_weight,
                                         self.beta)
        return (spec, amp, angle, time, energy, mr, das_reg, das_ce, ori_time, pred_time)
