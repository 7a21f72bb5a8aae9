"""Hash-grid encoding (HIP) — the `tcnn.Encoding(3, {"otype": "HashGrid", ...})`
the reference's networks call (model.py:66-68, 258-263).

tiny-cuda-nn is not vendored in the reference (requirements.txt:11 pins an
unversioned git URL), so this module follows upstream tiny-cuda-nn's
GridEncoding semantics and is checked against `oracle/hashgrid_oracle.py`
only: parity with tcnn itself is UNPINNED.

Semantics (per level l of L):
  scale_l = 2^(l*log2(per_level_scale)) * base_resolution - 1
  res_l   = ceil(scale_l) + 1
  size_l  = min(round_up(res_l^3, 8), 2^log2_hashmap_size)
  p = scale_l*x + 0.5; cell = floor(p); frac = p - cell
  index = dense (x + y*res + z*res^2) when res^3 <= size_l, else
          x*1 ^ y*2654435761 ^ z*805459861; then mod size_l
  out[l*2 + f] = sum over 8 corners of trilinear weight * table_l[index][f]
Parameters are kept as one fp32 vector (like tcnn's torch binding) and
initialised U(-1e-4, 1e-4).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .options import resolve
from .wcache import cast_weight
from ._lib import DTYPE_F16, DTYPE_F32


def level_layout(n_levels, log2_hashmap_size, base_resolution, per_level_scale=2.0):
    """(offsets[L+1] in entries, scale[L] fp32, res[L]) as tcnn computes them."""
    log2_pls = np.float32(math.log2(per_level_scale))
    offsets = [0]
    scales, res = [], []
    for l in range(n_levels):
        s = np.float32(np.exp2(np.float32(l) * log2_pls)) * np.float32(base_resolution) - np.float32(1.0)
        s = np.float32(s)
        r = int(math.ceil(float(s))) + 1
        dense = r ** 3 if float(r) ** 3 <= (2 ** 31 - 1) else 2 ** 31 - 1
        dense = (dense + 7) // 8 * 8
        size = min(dense, 1 << log2_hashmap_size)
        scales.append(float(s))
        res.append(r)
        offsets.append(offsets[-1] + size)
    return (np.array(offsets, dtype=np.int64), np.array(scales, dtype=np.float32),
            np.array(res, dtype=np.int32))


def _code(dtype):
    if dtype == torch.float32:
        return DTYPE_F32
    if dtype == torch.float16:
        return DTYPE_F16
    raise TypeError(f"hash grid supports float32/float16, got {dtype}")


class _HashGridFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, params, enc, cache=False):
        N = x.size(0)
        out = torch.empty(N, enc.n_output_dims, dtype=enc.dtype, device=x.device)
        st = torch.cuda.current_stream(x.device).cuda_stream
        table = enc.table(cache)
        _lib.call("avr_hashgrid_fwd", N, enc.n_levels, x.data_ptr(), table.data_ptr(),
                  _code(table.dtype), enc._off.ctypes.data, enc._scale.ctypes.data,
                  enc._res.ctypes.data, out.data_ptr(), _code(out.dtype), st)
        ctx.enc = enc
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        (x,) = ctx.saved_tensors
        enc = ctx.enc
        g = grad_out.contiguous()
        if g.dtype not in (torch.float32, torch.float16):
            g = g.float()
        st = torch.cuda.current_stream(x.device).cuda_stream
        N = x.size(0)
        mode = enc.options.hashgrid_bwd
        if mode == "atomic":
            gp = torch.zeros(enc.n_params, dtype=torch.float32, device=x.device)
            _lib.call("avr_hashgrid_bwd", N, enc.n_levels, x.data_ptr(), g.data_ptr(),
                      _code(g.dtype), enc._off.ctypes.data, enc._scale.ctypes.data,
                      enc._res.ctypes.data, gp.data_ptr(), st)
            return None, gp, None, None
        # partitioned (no global atomics), written rather than added: no
        # clearing pass over the table ("partitioned_add": the += form into
        # a cleared table, for A/B); workspace from the caching allocator
        add = mode == "partitioned_add"
        gp = (torch.zeros if add else torch.empty)(enc.n_params, dtype=torch.float32, device=x.device)
        nbytes = ctypes.c_int64()
        _lib.call("avr_hashgrid_bwd_workspace", N, enc.n_levels, enc._off.ctypes.data, ctypes.byref(nbytes))
        ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=x.device)
        _lib.call("avr_hashgrid_bwd_partitioned" if add else "avr_hashgrid_bwd_partitioned_set", N, enc.n_levels,
                  x.data_ptr(), g.data_ptr(),
                  _code(g.dtype), enc._off.ctypes.data, enc._scale.ctypes.data, enc._res.ctypes.data,
                  gp.data_ptr(), ws.data_ptr(), nbytes.value, st)
        return None, gp, None, None


class HashGridEncoding(nn.Module):
    """tcnn.Encoding(n_input_dims=3, encoding_config, dtype) replacement;
    `options` (avr_amd.KernelOptions) selects the backward's form."""

    def __init__(self, n_input_dims, encoding_config, dtype=None, seed=None, options=None):
        super().__init__()
        self.options = resolve(options)
        cfg = dict(encoding_config)
        if cfg.get("otype", "HashGrid") not in ("HashGrid", "Grid"):
            raise ValueError(f"unsupported encoding {cfg.get('otype')}")
        if n_input_dims != 3:
            raise ValueError("HashGridEncoding supports 3-D inputs")
        if int(cfg.get("n_features_per_level", 2)) != 2:
            raise ValueError("n_features_per_level must be 2")
        self.n_levels = int(cfg.get("n_levels", 16))
        self.log2_hashmap_size = int(cfg.get("log2_hashmap_size", 19))
        self.base_resolution = int(cfg.get("base_resolution", 16))
        self.per_level_scale = float(cfg.get("per_level_scale", 2.0))
        self.n_output_dims = 2 * self.n_levels
        self.dtype = torch.float16 if dtype is None else dtype
        # tcnn runs a module's forward on params cast to its precision
        # (Module.forward: self.params.to(param_precision)): fp16 tables for
        # fp16 encodings, the fp32 master copy receives the gradient
        self.param_dtype = torch.float16 if self.dtype == torch.float16 else torch.float32
        self._off, self._scale, self._res = level_layout(self.n_levels, self.log2_hashmap_size,
                                                         self.base_resolution, self.per_level_scale)
        self.n_params = int(self._off[-1]) * 2
        g = torch.Generator().manual_seed(1337 if seed is None else seed)
        init = (torch.rand(self.n_params, generator=g) * 2 - 1) * 1e-4
        self.params = nn.Parameter(init)

    def table(self, cache=False):
        """The level tables in the module's param precision."""
        return cast_weight(self.params, self.param_dtype, cache)

    def forward_level_major(self, x, unit_map=False):
        """Inference-only encoding with level-major output [L, N, 2]
        (`avr_hashgrid_fwd_lm`): the same values as forward(x) transposed.
        unit_map: x in [-1, 1] is encoded as (x + 1) / 2, the map applied on
        load (`avr_hashgrid_fwd_lm_unit`, bit-identical to mapping first)."""
        if not x.is_cuda:
            raise RuntimeError("HashGridEncoding needs a HIP tensor (no CPU fallback)")
        x = x.reshape(-1, 3).float().contiguous()
        N = x.size(0)
        out = torch.empty(self.n_levels, N, 2, dtype=self.dtype, device=x.device)
        st = torch.cuda.current_stream(x.device).cuda_stream
        table = self.table(not torch.is_grad_enabled())
        fn = "avr_hashgrid_fwd_lm_unit" if unit_map else "avr_hashgrid_fwd_lm"
        _lib.call(fn, N, self.n_levels, x.data_ptr(), table.data_ptr(),
                  _code(table.dtype), self._off.ctypes.data, self._scale.ctypes.data,
                  self._res.ctypes.data, out.data_ptr(), _code(out.dtype), st)
        return out

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("HashGridEncoding needs a HIP tensor (no CPU fallback)")
        x = x.reshape(-1, 3).float().contiguous()
        return _HashGridFn.apply(x, self.params, self, not torch.is_grad_enabled())
