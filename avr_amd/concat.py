"""Grouped feature concatenation (`csrc/concat.hip`) for the networks'
training path: the sigma-encoder and signal-network inputs of model.py:199-221
and 314-325, built in one pass from per-sample, per-ray and per-pose encodings
(each group's encoding read by its samples, not expanded), with a backward
that sums each group's gradient in fp32 in a fixed order."""
from __future__ import annotations

import ctypes

import torch

from . import _lib

_CODES = {torch.float32: _lib.DTYPE_F32, torch.float16: _lib.DTYPE_F16, torch.bfloat16: _lib.DTYPE_BF16}


class ConcatSrc(ctypes.Structure):
    """Mirror of `avr_concat_src` (include/avr_hip.h)."""

    _fields_ = [("data", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("dtype", ctypes.c_int32),
                ("rows_div", ctypes.c_int32), ("width", ctypes.c_int32), ("split", ctypes.c_int32)]


def _table(ptrs, grads, dtypes, divs, widths, splits):
    arr = (ConcatSrc * len(ptrs))()
    for i in range(len(ptrs)):
        arr[i].data = ptrs[i]
        arr[i].grad = grads[i]
        arr[i].dtype = _CODES[dtypes[i]]
        arr[i].rows_div = divs[i]
        arr[i].width = widths[i]
        arr[i].split = splits[i]
    return arr


class _GroupedConcat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, N, out_dtype, divs, splits, *parts):
        dev = parts[0].device
        width = sum(int(p.size(1)) for p in parts)
        out = torch.empty(N, width, dtype=out_dtype, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        tab = _table([p.data_ptr() for p in parts], [None] * len(parts), [p.dtype for p in parts], divs,
                     [int(p.size(1)) for p in parts], splits)
        _lib.call("avr_concat_fwd", N, len(parts), tab, out.data_ptr(), _CODES[out_dtype], st)
        ctx.meta = (N, divs, splits, [(tuple(p.shape), p.dtype) for p in parts])
        return out

    @staticmethod
    def backward(ctx, g):
        N, divs, splits, shapes = ctx.meta
        g = g.contiguous()
        dev = g.device
        grads = [torch.empty(shp, dtype=dt, device=dev) if ctx.needs_input_grad[4 + i] else None
                 for i, (shp, dt) in enumerate(shapes)]
        ws_floats = max([N // (d // sp) * shp[1] for (shp, _), d, sp in zip(shapes, divs, splits)
                         if sp > 1 and d > 1] or [0])
        ws = torch.empty(max(ws_floats, 1), dtype=torch.float32, device=dev)
        src = _table([None] * len(shapes), [None if gr is None else gr.data_ptr() for gr in grads],
                     [dt for _, dt in shapes], divs, [shp[1] for shp, _ in shapes], splits)
        st = torch.cuda.current_stream(dev).cuda_stream
        _lib.call("avr_concat_bwd", N, len(shapes), src, g.data_ptr(), _CODES[g.dtype], ws.data_ptr(), st)
        return (None, None, None, None, *grads)


def grouped_concat(parts, N, out_dtype, splits=None):
    """parts = [(tensor [N / rows_div, width], rows_div)] -> [N, sum widths]
    in out_dtype; `splits[i]` > 1 sums that part's gradient in two passes
    (rows_div / split rows, then split partial rows: per-pose groups)."""
    tensors = [t.contiguous() for t, _ in parts]
    divs = tuple(int(d) for _, d in parts)
    for t, d in zip(tensors, divs):
        if t.size(0) * d != N:
            raise ValueError(f"part of {t.size(0)} rows x rows_div {d} != {N} samples")
        if t.data_ptr() % 16 or t.size(1) % 8:
            raise ValueError("parts must be 16-byte aligned with widths a multiple of 8")
    sp = tuple(int(s) for s in (splits or [1] * len(parts)))
    return _GroupedConcat.apply(int(N), out_dtype, divs, sp, *tensors)
