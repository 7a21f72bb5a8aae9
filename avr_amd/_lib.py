"""ctypes binding of the HIP C-ABI (`include/avr_hip.h`, `libavr_hip.so`).

The product path has no CPU fallback: if the library is missing or a GPU is
not available, every render call raises.  The library is built in-tree by
`__graft_entry__.build()` (make -C avr_amd/csrc).
"""
from __future__ import annotations

import ctypes
import math
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libavr_hip.so")

DTYPE_F32 = 0
DTYPE_F16 = 1
DTYPE_BF16 = 2
MAX_AZI = 512  # AVR_MAX_AZI

_c_i32 = ctypes.c_int32
_c_i64 = ctypes.c_int64
_c_f32 = ctypes.c_float
_vp = ctypes.c_void_p


class RenderParams(ctypes.Structure):
    """Mirror of `avr_render_params` (include/avr_hip.h)."""

    _fields_ = [
        ("n_azi", _c_i32),
        ("n_ele", _c_i32),
        ("n_samples", _c_i32),
        ("T", _c_i32),
        ("n_rays", _c_i32),
        ("depth_scale", _c_f32),
        ("depth_offset", _c_f32),
        ("lo", _c_f32),
        ("span", _c_f32),
        ("fs", _c_f32),
        ("speed", _c_f32),
        ("pathloss", _c_f32),
        ("azi_jitter", _c_f32),
        ("two_pi", _c_f32),
        ("phase_c", _c_f32),
        ("near_clamp", _c_i32),
        ("pl_len", _c_i32),
    ]

    def key(self):
        """Hashable value of every field (computed once: render_params builds
        a fresh object and nothing mutates it afterwards)."""
        k = self.__dict__.get("_key")
        if k is None:
            k = self._key = tuple(getattr(self, f) for f, _ in self._fields_)
        return k


def _f32(x) -> float:
    return float(np.float32(x))


def render_params(cfg: dict, T: int, n_rays: int | None = None) -> RenderParams:
    """Round the `render:` scalars exactly as the reference's torch ops do.

    Python evaluates the scalar sub-expressions in double (renderer.py:54,
    97, 98, 108, 128, 149) and torch rounds the result to fp32 at the op.
    """
    p = RenderParams()
    p.n_azi = int(cfg["n_azi"])
    p.n_ele = int(cfg["n_ele"])
    p.n_samples = int(cfg["n_samples"])
    p.T = int(T)
    p.n_rays = p.n_azi * p.n_ele + 2 if n_rays is None else int(n_rays)
    p.depth_scale = _f32(cfg["far"] - cfg["near"])
    p.depth_offset = _f32(cfg["near"])
    p.lo = _f32(cfg["xyz_min"])
    p.span = _f32(cfg["xyz_max"] - cfg["xyz_min"])
    p.fs = _f32(cfg["fs"])
    p.speed = _f32(cfg["speed"])
    p.pathloss = _f32(cfg["pathloss"])
    p.azi_jitter = _f32(np.pi * 2 / cfg["n_azi"])
    p.two_pi = _f32(np.pi * 2)
    p.phase_c = _f32((-2 * np.pi) / T)
    p.near_clamp = int(0.1 / cfg["speed"] * cfg["fs"])
    p.pl_len = int(math.ceil(T * 2.5))
    return p


class TablePtrs(ctypes.Structure):
    """Mirror of `avr_table_ptrs` (include/avr_hip.h)."""

    _fields_ = [("d_vals", ctypes.c_void_p), ("shift", ctypes.c_void_p),
                ("pl_table", ctypes.c_void_p), ("phase", ctypes.c_void_p),
                ("twiddle", ctypes.c_void_p), ("ir_twiddle", ctypes.c_void_p)]


_SIGS = {
    "avr_last_error": (ctypes.c_char_p, []),
    "avr_abi_version": (ctypes.c_int, []),
    "avr_pinned_alloc": (ctypes.c_int, [_c_i64, _vp, _vp]),
    "avr_pinned_free": (ctypes.c_int, [_vp]),
    "avr_graph_launch": (ctypes.c_int, [_vp, _vp]),
    "avr_tables": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "avr_depth_samples": (ctypes.c_int, [_vp, _vp, _vp]),
    "avr_ir_twiddle": (ctypes.c_int, [_c_i32, _vp, _vp]),
    "avr_ray_directions": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "avr_sample_points": (ctypes.c_int, [_vp, _c_i32] + [_vp] * 10),
    "avr_sample_rays": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32] + [_vp] * 9),
    "avr_weights_fwd": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32] + [_vp] * 7),
    "avr_ray_reduce_fwd": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_sample_rays_dev": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32] + [_vp] * 9),
    "avr_sample_rays_staged": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32, _c_i32] + [_vp] * 7),
    "avr_reduce_splits": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp]),
    "avr_dft_phase_fwd": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32, _vp, _vp, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_spectrum_finalize": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _vp, _vp, _vp]),
    "avr_irfft": (ctypes.c_int, [_c_i32, _c_i32, _vp, _vp, _vp, _vp]),
    "avr_irfft_bwd": (ctypes.c_int, [_c_i32, _c_i32, _vp, _vp, _vp, _vp]),
    "avr_dft_phase_bwd": (ctypes.c_int, [_vp, _c_i32] + [_vp] * 7),
    "avr_ray_reduce_bwd": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32] + [_vp] * 6),
    "avr_weights_bwd": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32, _vp, _vp, _vp, _vp]),
    "avr_hashgrid_fwd": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _c_i32, _vp]),
    "avr_hashgrid_fwd_lm": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _c_i32, _vp]),
    "avr_hashgrid_fwd_lm_unit": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _c_i32, _vp]),
    "avr_ray_pose_bias": (ctypes.c_int, [_c_i32, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp,
                                         _c_i32, _vp, _vp, _vp, _vp, _c_i32, _c_i32, _c_i32, _vp, _vp,
                                         _c_i32, _vp, _vp]),
    "avr_hashgrid_bwd": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _vp]),
    "avr_hashgrid_bwd_workspace": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp]),
    "avr_hashgrid_bwd_partitioned": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _vp,
                                                    _c_i64, _vp]),
    "avr_hashgrid_bwd_partitioned_set": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _vp,
                                                    _c_i64, _vp]),
    "avr_linear_wgrad_splits": (ctypes.c_int, [_c_i64, _c_i32, _c_i32, _vp]),
    "avr_linear512_pack_w2": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _vp]),
    "avr_linear512_mask_fwd": (ctypes.c_int, [_c_i64, _vp, _vp, _c_i32, _vp, _vp, _vp]),
    "avr_linear_wgrad": (ctypes.c_int, [_c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_linear_out1_fwd": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_narrow_mm": (ctypes.c_int, [_c_i64, _c_i32, _c_i32, _vp, _vp, _c_i32, _c_i32, _vp, _vp, _vp]),
    "avr_linear_out1_workspace": (ctypes.c_int, [_c_i32, _vp]),
    "avr_linear_out1_bwd": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp]),
    "avr_head_splits": (ctypes.c_int, [_vp, _c_i32, _c_i32, _c_i32, _vp]),
    "avr_head_sort": (ctypes.c_int, [_vp, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "avr_head_pack_w": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _c_i32, _vp, _vp]),
    "avr_head_exact_layout": (ctypes.c_int, [_vp, _c_i32, _c_i32, _c_i32, _vp, _vp]),
    "avr_head_pack_w_exact": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32, _vp, _vp]),
    "avr_head_fwd_exact": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _c_i32,
                                          _vp, _vp, _vp]),
    "avr_head_fwd": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _c_i32, _vp,
                                    _vp]),
    "avr_head_bwd_workspace": (ctypes.c_int, [_vp, _c_i32, _c_i32, _c_i32, _vp]),
    "avr_head_bwd": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _c_i64, _vp]),
    "avr_head_bwd2": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                     _c_i32, _vp, _vp, _vp, _vp, _c_i64, _vp]),
    "avr_criterion_window_len": (ctypes.c_int, []),
    "avr_criterion_workspace": (ctypes.c_int, [_c_i32, _c_i32, _vp]),
    "avr_criterion_fwd": (ctypes.c_int, [_c_i32, _c_i32] + [_vp] * 10 + [_c_i64, _vp]),
    "avr_criterion_fwd2": (ctypes.c_int, [_c_i32, _c_i32] + [_vp] * 11 + [_c_i64, _vp]),
    "avr_criterion_bwd": (ctypes.c_int, [_c_i32, _c_i32] + [_vp] * 11 + [_c_i64, _vp, _vp]),
    "avr_das_workspace": (ctypes.c_int, [_vp]),
    "avr_das_fwd": (ctypes.c_int, [_c_i32] + [_vp] * 5 + [_c_f32] * 3 + [_vp, _vp, _c_i64, _vp]),
    "avr_das_bwd": (ctypes.c_int, [_c_i32] + [_vp] * 3 + [_c_f32] * 3 + [_vp, _vp, _c_i64, _vp, _vp]),
    "avr_scale_sanitize": (ctypes.c_int, [_c_i32, _vp, _vp, _vp, _vp]),
    "avr_grad_clip_workspace": (ctypes.c_int, [_c_i32, _vp, _vp]),
    "avr_grad_clip_coef": (ctypes.c_int, [_c_i32, _vp, _vp, ctypes.c_float, _vp, ctypes.c_int64, _vp, _vp, _vp]),
    "avr_adam_step": (ctypes.c_int, [_c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_float, ctypes.c_float, _vp, _vp]),
    "avr_concat_fwd": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp]),
    "avr_concat_bwd": (ctypes.c_int, [_c_i64, _c_i32, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_sigma_pack_bytes": (ctypes.c_int, [_c_i32, _vp]),
    "avr_sigma_desc_size": (ctypes.c_int, []),
    "avr_sigma_fwd": (ctypes.c_int, [_vp] * 3 + [_c_i32, _vp, _vp]),
    "avr_render_core_layout": (ctypes.c_int, [_vp, _c_i32, _c_i32, _vp, _vp]),
    "avr_render_core_fwd": (ctypes.c_int, [_vp, _c_i32, _vp, _c_i32, _vp, _c_i32] + [_vp] * 5
                            + [_c_i64] + [_vp] * 5),
}

EXPORTS = tuple(_SIGS)

# entry points of the shapes build only (include/avr_hip.h, AVR_SHAPE_PROBES):
# typed when a tool loads that library in place of the product one
_SHAPES_SIGS = {
    "avr_linear512_pack_w": (ctypes.c_int, [_vp, _c_i32, _vp, _vp]),
    "avr_linear512_relu_fwd": (ctypes.c_int, [_c_i64, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_mlp512x2_pack_w": (ctypes.c_int, [_vp, _vp, _c_i32, _vp, _vp]),
    "avr_mlp512x2_fwd": (ctypes.c_int, [_c_i64, _vp, _vp, _c_i32, _vp, _vp]),
    "avr_linear_pack_w": (ctypes.c_int, [_c_i32, _c_i32, _vp, _c_i32, _vp, _vp]),
}

_lock = threading.Lock()
_lib = None


def load():
    """Load libavr_hip.so once; raise with a clear message if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"avr_amd: HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C avr_amd/csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in _SHAPES_SIGS.items():
            if hasattr(lib, name):
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
        if lib.avr_abi_version() != 2:
            raise RuntimeError("avr_amd: libavr_hip.so ABI version mismatch")
        _lib = lib
        return lib


def call(name: str, *args):
    """Invoke a C-ABI entry point and raise RuntimeError on a nonzero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.avr_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")
