"""Delay-and-sum direction losses (utils/criterion.py:35-67, 100-122) on the GPU.

Used by `avr_amd.criterion.Criterion` when `das_reg_loss_weight` or
`das_ce_loss_weight` is positive (the 8-channel real-environment configs,
e.g. avr_real_exp_ch_emb_add_das_optuna.yml).  Inputs are the criterion's
pred_time / ori_time [8, n]; the kernels are in `csrc/das.hip`
(`avr_das_fwd` / `avr_das_bwd`), and the gradient flows back into pred_time
and from there through the criterion's adjoint irfft.
"""
from __future__ import annotations

import ctypes
import math
import threading

import torch

from . import _lib
from .renderer import _ir_twiddle

_N_FFT = 512   # criterion.py:43
_MICS = 8      # criterion.py:41
_TABLES: dict = {}
_LOCK = threading.Lock()
_WS_BYTES = None


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _steering(dev, fs, speed):
    """steer [360][8][257] complex64 and theta [360], built with the
    reference's own torch ops on the CPU (criterion.py:24, 45-60) once per
    (device, fs, speed)."""
    key = (dev.index, float(fs), float(speed))
    t = _TABLES.get(key)
    if t is None:
        with _LOCK:
            t = _TABLES.get(key)
            if t is None:
                angles = torch.deg2rad(torch.arange(0.0, 360.0, 1.0))
                freqs = torch.fft.rfftfreq(_N_FFT, 1 / fs)
                mic_angles = torch.linspace(math.pi / 2, math.pi / 2 + 2 * math.pi, _MICS + 1)[:-1]
                mic_pos = torch.stack([torch.cos(mic_angles), torch.sin(mic_angles)], dim=-1)
                mic_pos -= mic_pos.mean(dim=0)
                steer = torch.zeros(len(angles), _MICS, freqs.numel(), dtype=torch.cfloat)
                for i, theta in enumerate(angles):
                    u = torch.tensor([torch.cos(theta), torch.sin(theta)])
                    delays = (mic_pos @ u) / speed
                    steer[i] = torch.exp(-1j * 2 * math.pi * delays[:, None] * freqs[None, :])
                t = (torch.view_as_real(steer).contiguous().to(dev), angles.float().to(dev))
                _TABLES[key] = t
    return t


def _ws_bytes():
    global _WS_BYTES
    if _WS_BYTES is None:
        out = ctypes.c_int64(0)
        _lib.call("avr_das_workspace", ctypes.byref(out))
        _WS_BYTES = int(out.value)
    return _WS_BYTES


class _DasFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred_time, ori_time, fs, speed, beta, w_reg, w_ce):
        dev = pred_time.device
        n = pred_time.size(1)
        steer, angles = _steering(dev, fs, speed)
        tw = _ir_twiddle(_N_FFT, dev)
        nbytes = _ws_bytes()
        ws = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        losses = torch.empty(2, dtype=torch.float32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        with torch.cuda.device(dev):
            _lib.call("avr_das_fwd", n, _ptr(pred_time), _ptr(ori_time), _ptr(steer),
                      _ptr(angles), _ptr(tw), ctypes.c_float(beta), ctypes.c_float(w_reg),
                      ctypes.c_float(w_ce), _ptr(losses), _ptr(ws), nbytes, stream)
        ctx.save_for_backward(ws)
        ctx.cfg = (n, fs, speed, beta, w_reg, w_ce)
        ctx.set_materialize_grads(False)
        return losses[0], losses[1]

    @staticmethod
    def backward(ctx, g_reg, g_ce):
        (ws,) = ctx.saved_tensors
        n, fs, speed, beta, w_reg, w_ce = ctx.cfg
        if g_reg is None and g_ce is None:
            return (None,) * 7
        dev = ws.device
        zero = torch.zeros((), dtype=torch.float32, device=dev)
        g = torch.stack([(zero if g_reg is None else g_reg.reshape(()).float()),
                         (zero if g_ce is None else g_ce.reshape(()).float())])
        steer, angles = _steering(dev, fs, speed)
        grad = torch.empty(_MICS, n, dtype=torch.float32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        with torch.cuda.device(dev):
            _lib.call("avr_das_bwd", n, _ptr(steer), _ptr(angles), _ptr(_ir_twiddle(_N_FFT, dev)),
                      ctypes.c_float(beta), ctypes.c_float(w_reg), ctypes.c_float(w_ce), _ptr(g),
                      _ptr(ws), ws.numel() * 4, _ptr(grad), stream)
        return grad, None, None, None, None, None, None


def das_losses(pred_time, ori_time, fs, speed, reg_weight, ce_weight, beta=100.0):
    """(das_reg_loss, das_ce_loss) of criterion.py:100-122 for 8 channels."""
    M = pred_time.shape[0]
    assert M == _MICS, f"Expected 8 microphones, but got {M}"
    if not pred_time.is_cuda:
        raise RuntimeError("avr_amd.das needs HIP tensors (no CPU fallback)")
    return _DasFn.apply(pred_time.float().contiguous(), ori_time.detach().float().contiguous(),
                        float(fs), float(speed), float(beta), float(reg_weight), float(ce_weight))
