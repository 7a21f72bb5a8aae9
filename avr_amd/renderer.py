"""Drop-in `AVRRender` for MI355X: the reference's renderer interface, HIP inside.

Mirrors `renderer.py` of the reference (KMASAHIRO/AVR):

* `AVRRender(networks_fn, **render_cfg)` — renderer.py:13-29, reads
  n_samples, near, far, n_azi, n_ele, speed, fs, pathloss, xyz_min, xyz_max
  and ignores extra keys (e.g. `sig_length`, avr_raf_furnished.yml:22).
* `forward(rays_o, position_tx, direction_tx=None, ch_idx=None) -> [B, F, 2]`
  — renderer.py:31-124.  `ch_idx` is passed to `network_fn` only when it is
  not None (the reference always passes it, which `AVRModel_complex.forward`
  (model.py:291) rejects).
* module functions `ray_directions`, `normalize_points`,
  `denormalize_points` with the reference's names (renderer.py:127-165).

Everything after the network call runs in hand-written HIP kernels
(`avr_amd/csrc`) through the C-ABI; autograd flows to the network's `attn`
and `signal` outputs through `RenderCore`.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math
import threading

import torch
import torch.nn as nn

from . import _lib
from ._lib import DTYPE_BF16, DTYPE_F16, DTYPE_F32, render_params
from .options import tuning_env
from .wcache import cache_lookup, cache_store, capturing, cast_weight


_RENDER_KEYS = ("n_samples", "near", "far", "n_azi", "n_ele", "speed", "fs", "pathloss",
                "xyz_min", "xyz_max")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(device):
    return torch.cuda.current_stream(device).cuda_stream


class _NoGuard:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_GUARD = _NoGuard()


def _on(dev):
    """torch.cuda.device(dev), skipped when dev is already current (the
    common case: entering the guard costs more host time than a launch)."""
    return _NO_GUARD if torch.cuda.current_device() == dev.index else torch.cuda.device(dev)


def _f32_on(t, dev):
    """t as a contiguous fp32 tensor on dev (no-op calls skipped: each costs
    host time on the latency path)."""
    if t.device != dev or t.dtype != torch.float32:
        t = t.to(dev, torch.float32)
    return t if t.is_contiguous() else t.contiguous()


def _dtype_code(t):
    if t.dtype == torch.float32:
        return DTYPE_F32
    if t.dtype == torch.float16:
        return DTYPE_F16
    if t.dtype == torch.bfloat16:
        return DTYPE_BF16
    raise TypeError(f"unsupported dtype {t.dtype} (float32, float16 or bfloat16)")


# --------------------------------------------------------------------------
# per-device, per-config resident tables (pose independent)
# --------------------------------------------------------------------------
class Tables:
    """d_vals, frac, shift, path-loss table, phase[S,F], twiddles on one device."""

    def __init__(self, p, device):
        S, T = p.n_samples, p.T
        F = T // 2 + 1
        f32 = dict(dtype=torch.float32, device=device)
        self.d_vals = torch.empty(S, **f32)
        self.frac = torch.empty(S, **f32)
        self.shift = torch.empty(S, dtype=torch.int32, device=device)
        self.pl = torch.empty(p.pl_len, **f32)
        self.phase = torch.empty(S, F, 2, **f32)
        self.twiddle = torch.empty(T, 2, **f32)
        n = 2 * (F - 1)
        self.ir_n = n
        self.ir_twiddle = torch.empty(max(n, 2), 2, **f32)
        st = _stream(device)
        with torch.cuda.device(device):
            _lib.call("avr_tables", ctypes_ref(p), _ptr(self.d_vals), _ptr(self.frac),
                      _ptr(self.shift), _ptr(self.pl), _ptr(self.phase), _ptr(self.twiddle), st)
            if n >= 2:
                _lib.call("avr_ir_twiddle", n, _ptr(self.ir_twiddle), st)
        # shift values are needed on the host for the reference's range check
        shifts = self.shift.cpu()
        self.max_shift = int(shifts.max().item()) if S > 0 else 0
        self.ptrs = _lib.TablePtrs(self.d_vals.data_ptr(), self.shift.data_ptr(),
                                   self.pl.data_ptr(), self.phase.data_ptr(),
                                   self.twiddle.data_ptr(),
                                   self.ir_twiddle.data_ptr() if n >= 2 else None)
        self._layouts = {}

    def core_layout(self, p, B, sig_code):
        """(offsets[5], n_split, k_split) of avr_render_core_fwd's workspace."""
        # tuning overrides read by the library (options.TUNING_ENV) are part of the key
        key = (p.n_rays, B, sig_code) + tuning_env()
        v = self._layouts.get(key)
        if v is None:
            with _TABLE_LOCK:
                v = self._layouts.get(key)
                if v is None:
                    off = (ctypes.c_int64 * 5)()
                    sp = (ctypes.c_int32 * 2)()
                    _lib.call("avr_render_core_layout", ctypes_ref(p), B, sig_code, off, sp)
                    v = (tuple(off), int(sp[0]), int(sp[1]))
                    self._layouts[key] = v
        return v


def ctypes_ref(p):
    import ctypes

    return ctypes.byref(p)


_TABLE_CACHE: dict = {}
_TABLE_LOCK = threading.RLock()


def get_tables(p, device) -> Tables:
    key = (device.index, p.key())
    t = _TABLE_CACHE.get(key)
    if t is None:
        with _TABLE_LOCK:
            t = _TABLE_CACHE.get(key)
            if t is None:
                t = Tables(p, device)
                _TABLE_CACHE[key] = t
    return t


def check_config(p, tables: Tables):
    """Reference-equivalent constraints (renderer.py:96-100)."""
    if p.near_clamp + 1 >= p.pl_len:
        raise IndexError("path_loss[prev_part+1] out of range (renderer.py:99): "
                         f"int(0.1/speed*fs)+1 = {p.near_clamp + 1} >= {p.pl_len}")
    if tables.max_shift + p.T > p.pl_len:
        raise RuntimeError(
            "stack expects each tensor to be equal size: receiver delay "
            f"{tables.max_shift} samples + T={p.T} exceeds the path-loss table ({p.pl_len}); "
            "the reference fails the same way at renderer.py:100 (needs shift <= 1.5T)")


# --------------------------------------------------------------------------
# launch heuristics
# --------------------------------------------------------------------------
def reduce_splits(p, B, sig_code):
    """Ray splits of the reduction, decided by the library for this shape."""
    import ctypes

    n = ctypes.c_int32(0)
    _lib.call("avr_reduce_splits", ctypes_ref(p), B, sig_code, ctypes.byref(n))
    return int(n.value)


def pick_k_split(B, S, T):
    """t-slices of the DFT GEMM: about 256 workgroups. AVR_KSPLIT overrides."""
    F = T // 2 + 1
    nkc = math.ceil(T / 64)
    forced = tuning_env()[1]
    forced = int(forced) if forced else None
    if forced:
        return max(1, min(nkc, forced))
    base = math.ceil(F / 128) * math.ceil(S / 32) * B
    return max(1, min(nkc, math.ceil(256 / max(1, base))))


# --------------------------------------------------------------------------
# autograd core: (attn, signal) -> spectrum
# --------------------------------------------------------------------------
def _weights(p, attn, rays_o, position_tx, dirs, tables, st):
    """avr_weights_fwd: compositing weights w and source delays [B, R, S]."""
    B = attn.size(0)
    R, S = p.n_rays, p.n_samples
    dev = attn.device
    w = torch.empty(B, R, S, dtype=torch.float32, device=dev)
    delay = torch.empty(B, R, S, dtype=torch.int32, device=dev)
    _lib.call("avr_weights_fwd", ctypes_ref(p), B, _ptr(attn), _dtype_code(attn), _ptr(rays_o),
              _ptr(position_tx), _ptr(dirs), _ptr(tables.d_vals), _ptr(w), _ptr(delay), st)
    return w, delay


def _spectrum(p, tables, part, n_split, B, dev, st):
    """Partials [n_split, B, S, T] -> DFT + phase -> [B, F, 2]."""
    S, T = p.n_samples, p.T
    F = T // 2 + 1
    k_split = pick_k_split(B, S, T)
    P = math.ceil(S / 32) * k_split
    spart = torch.empty(B, P, F, 2, dtype=torch.float32, device=dev)
    _lib.call("avr_dft_phase_fwd", ctypes_ref(p), B, _ptr(part), n_split, _ptr(tables.pl),
              _ptr(tables.shift), _ptr(tables.phase), _ptr(tables.twiddle), k_split,
              _ptr(spart), st)
    out = torch.empty(B, F, 2, dtype=torch.float32, device=dev)
    _lib.call("avr_spectrum_finalize", B, P, F, _ptr(spart), _ptr(out), st)
    return out


def _grad_z(p, tables, grad_out, B, dev, st):
    """avr_dft_phase_bwd: dL/dz [B, S, T] (path loss and tail mask included)."""
    g = grad_out.contiguous().float()
    gz = torch.empty(B, p.n_samples, p.T, dtype=torch.float32, device=dev)
    _lib.call("avr_dft_phase_bwd", ctypes_ref(p), B, _ptr(g), _ptr(tables.pl), _ptr(tables.shift),
              _ptr(tables.phase), _ptr(tables.twiddle), _ptr(gz), st)
    return gz


def _grad_attn(p, tables, attn, grad_w, st):
    grad_attn = torch.empty_like(attn)
    _lib.call("avr_weights_bwd", ctypes_ref(p), attn.size(0), _ptr(attn), _dtype_code(attn),
              _ptr(tables.d_vals), _ptr(grad_w), _ptr(grad_attn), st)
    return grad_attn


def _render_core_fwd(attn, signal, p, tables, rays_o, position_tx, dirs, ir_out, timer=None):
    """avr_render_core_fwd -> (out [B, F, 2], workspace, layout offsets).

    `timer` (bench.py / tools/tune.py instrumentation, normally None) hands
    out a pair of hipEvent_t the library records around the ray-reduction
    launch on its stream."""
    dev = signal.device
    B = signal.size(0)
    F = p.T // 2 + 1
    sig_code = _dtype_code(signal)
    off, n_split, _ = tables.core_layout(p, B, sig_code)
    ws = torch.empty(off[4], dtype=torch.uint8, device=dev)
    out = torch.empty(B, F, 2, dtype=torch.float32, device=dev)
    ev0 = ev1 = None
    if timer is not None:
        R, S = p.n_rays, p.n_samples
        delay = ws[off[1]:off[1] + B * R * S * 4].view(torch.int32).view(B, R, S)
        ev0, ev1 = timer.events(n_split=n_split, delay=delay, shift=tables.shift)
    _lib.call("avr_render_core_fwd", ctypes_ref(p), B, _ptr(attn), _dtype_code(attn),
              _ptr(signal), sig_code, _ptr(rays_o), _ptr(position_tx), _ptr(dirs),
              ctypes.byref(tables.ptrs), _ptr(ws), off[4], _ptr(out), _ptr(ir_out), ev0, ev1,
              _stream(dev))
    return out, ws, off


class RenderCore(torch.autograd.Function):
    """Everything after the network call (renderer.py:75-121) as HIP kernels.

    Inputs: attn [B, R*S] and signal [B, R*S, T] (fp32, fp16 or bf16,
    contiguous), plus the pose geometry.  Output [B, F, 2] fp32.  Gradients
    flow to attn and signal (poses are constants, as in the reference).
    """

    @staticmethod
    def forward(ctx, attn, signal, p, tables, rays_o, position_tx, dirs, ir_out=None, timer=None):
        """One native call (avr_render_core_fwd): weights, ray reduction, DFT
        + phase, finalize, and the irfft into `ir_out` [B, 2(F-1)] when given
        (forward only, as spectrum_to_ir)."""
        out, ws, off = _render_core_fwd(attn, signal, p, tables, rays_o, position_tx, dirs, ir_out, timer)
        B, R, S = signal.size(0), p.n_rays, p.n_samples
        w = ws[off[0]:off[0] + B * R * S * 4].view(torch.float32).view(B, R, S)
        delay = ws[off[1]:off[1] + B * R * S * 4].view(torch.int32).view(B, R, S)
        ctx.p, ctx.tables = p, tables
        ctx.save_for_backward(attn, signal, w, delay)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        attn, signal, w, delay = ctx.saved_tensors
        p, tables = ctx.p, ctx.tables
        dev = signal.device
        B = signal.size(0)
        R, S = p.n_rays, p.n_samples
        st = _stream(dev)
        gz = _grad_z(p, tables, grad_out, B, dev, st)
        grad_signal = torch.empty_like(signal)
        grad_w = torch.empty(B, R, S, dtype=torch.float32, device=dev)
        _lib.call("avr_ray_reduce_bwd", ctypes_ref(p), B, _ptr(signal), _dtype_code(signal),
                  _ptr(gz), _ptr(w), _ptr(delay), _ptr(grad_signal), _ptr(grad_w), st)
        grad_attn = _grad_attn(p, tables, attn, grad_w, st) if ctx.needs_input_grad[0] else None
        return (grad_attn, grad_signal if ctx.needs_input_grad[1] else None,
                None, None, None, None, None, None, None)


def _packed_head_weight(w_master, W, cache, pref, shape_key, st):
    """W in avr_head_fwd's block-major layout (avr_head_pack_w).  With
    `cache` (no autograd graph recorded) the copy is kept on the master
    weight until it changes, like wcache.cast_weight."""
    key = (W.data_ptr(), w_master._version, shape_key)
    cache = cache and not capturing()
    if cache:
        hit = cache_lookup(w_master, "_avr_headpack", key)
        if hit is not None:
            return hit
    B, K, code = shape_key[2], shape_key[3], shape_key[4]
    Wp = torch.empty_like(W)
    _lib.call("avr_head_pack_w", pref, B, K, _ptr(W), code, _ptr(Wp), st)
    return cache_store(w_master, "_avr_headpack", key, Wp) if cache else Wp


def _packed_exact_weight(w_master, W, cache, pref, shape_key, nbytes, st):
    """W in the exact head's MFMA-fragment order (avr_head_pack_w_exact),
    cached on the master weight like _packed_head_weight."""
    key = (W.data_ptr(), w_master._version, shape_key)
    cache = cache and not capturing()
    if cache:
        hit = cache_lookup(w_master, "_avr_exactpack", key)
        if hit is not None:
            return hit
    K, code = shape_key[1], shape_key[2]
    Wf = torch.empty(nbytes // 2, dtype=W.dtype, device=W.device)
    _lib.call("avr_head_pack_w_exact", pref, K, _ptr(W), code, _ptr(Wf), st)
    return cache_store(w_master, "_avr_exactpack", key, Wf) if cache else Wf


class FusedHeadCore(torch.autograd.Function):
    """Render core with the signal network's last linear layer folded in
    (kernels in csrc/head.hip).

    Inputs: attn [B, R*S], the last hidden activation h [B, R*S, K] and the
    layer's fp32 master weight [T, K] (cast to `dtype`, fp32 or bf16, as the
    unfused layer would).  Equal to RenderCore on signal = h @ W^T, without
    the [B, R*S, T] tensor, the R*S*K*T GEMM or their backward; gradients to
    attn, h and the weight.
    """

    @staticmethod
    def forward(ctx, attn, h, w_master, dtype, p, tables, rays_o, position_tx, dirs, cache=False, exact=False,
                relu_h=False, timer=None):
        dev = h.device
        B, K = h.size(0), h.size(-1)
        S, T = p.n_samples, p.T
        st = _stream(dev)
        pref = ctypes_ref(p)
        W = cast_weight(w_master, dtype, cache)
        code = _dtype_code(h)
        w, delay = _weights(p, attn, rays_o, position_tx, dirs, tables, st)
        R = p.n_rays
        perm = torch.empty(B, S, R, dtype=torch.int32, device=dev)
        ws = torch.empty(B, S, R, dtype=torch.float32, device=dev)
        cnt = torch.empty(B, S, T, dtype=torch.int32, device=dev)
        _lib.call("avr_head_sort", pref, B, _ptr(w), _ptr(delay), _ptr(perm), _ptr(ws), _ptr(cnt), st)
        if exact:
            # every signal element formed and rounded to the 16-bit type, as
            # the unfused layer (the reference network) outputs it
            ns, wbytes = ctypes.c_int32(0), ctypes.c_int64(0)
            _lib.call("avr_head_exact_layout", pref, B, K, code, ctypes.byref(ns), ctypes.byref(wbytes))
            n_split = ns.value
            part = torch.empty(n_split, B, S, T, dtype=torch.float32, device=dev)
            queue = torch.empty(256, dtype=torch.int32, device=dev)  # work-queue counters (zeroed by the call)
            Wf = _packed_exact_weight(w_master, W, cache, pref, (p.T, K, code), wbytes.value, st)
            # (bench.py's timer: events around the head on its stream, torch's current one)
            ev0, ev1 = timer.head_events(delay, tables.shift, K) if timer is not None else (None, None)
            if ev0 is not None:
                ev0.record()
            _lib.call("avr_head_fwd_exact", pref, B, K, _ptr(h), _ptr(Wf), code, _ptr(perm), _ptr(ws), _ptr(cnt),
                      _ptr(delay), n_split, _ptr(part), _ptr(queue), st)
            if ev1 is not None:
                ev1.record()
        else:
            ns = ctypes.c_int32(0)
            _lib.call("avr_head_splits", pref, B, K, code, ctypes.byref(ns))
            n_split = ns.value
            part = torch.empty(n_split, B, S, T, dtype=torch.float32, device=dev)
            Wp = _packed_head_weight(w_master, W, cache, pref, (p.T, R, B, K, code), st)
            _lib.call("avr_head_fwd", pref, B, K, _ptr(h), _ptr(Wp), code, _ptr(perm), _ptr(ws), _ptr(cnt),
                      n_split, _ptr(part), st)
        out = _spectrum(p, tables, part, n_split, B, dev, st)
        ctx.p, ctx.tables, ctx.relu_h = p, tables, relu_h
        ctx.save_for_backward(attn, h, W, w, delay, perm, ws, cnt)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        attn, h, W, w, delay, perm, ws, cnt = ctx.saved_tensors
        p, tables = ctx.p, ctx.tables
        dev = h.device
        B, K = h.size(0), h.size(-1)
        R, S, T = p.n_rays, p.n_samples, p.T
        st = _stream(dev)
        pref = ctypes_ref(p)
        code = _dtype_code(h)
        gz = _grad_z(p, tables, grad_out, B, dev, st)
        nbytes = ctypes.c_int64(0)
        _lib.call("avr_head_bwd_workspace", pref, B, K, code, ctypes.byref(nbytes))
        work = torch.empty(max(1, nbytes.value // 4), dtype=torch.float32, device=dev)
        grad_h = torch.empty_like(h)
        grad_w = torch.empty(B, R, S, dtype=torch.float32, device=dev)
        grad_W = torch.empty(T, K, dtype=torch.float32, device=dev)
        # relu_h: grad_h leaves with h's ReLU backward applied (the layer
        # that produced h was told so through its link and skips its own)
        _lib.call("avr_head_bwd2", pref, B, K, _ptr(h), _ptr(W), code, _ptr(w), _ptr(delay), _ptr(perm),
                  _ptr(ws), _ptr(cnt), _ptr(gz), int(ctx.relu_h), _ptr(grad_h), _ptr(grad_w), _ptr(grad_W),
                  _ptr(work), nbytes.value, st)
        grad_attn = _grad_attn(p, tables, attn, grad_w, st) if ctx.needs_input_grad[0] else None
        return (grad_attn, grad_h if ctx.needs_input_grad[1] else None,
                grad_W if ctx.needs_input_grad[2] else None, None, None, None, None, None, None, None, None, None,
                None)


def _poison_nonfinite(out, tensors, ir_out=None):
    """out + NaN where any element of `tensors` is non-finite, else out + 0
    (the reference's NaN propagation through its masks; no host sync)."""
    bad = None
    for t in tensors:
        b = ~torch.isfinite(t).all()
        bad = b if bad is None else bad | b
    # scalar operands: no host-to-device copy, so a HIP-graph capture of a
    # render with this option stays valid
    poison = torch.where(bad, float("nan"), 0.0)
    if ir_out is not None:
        ir_out.add_(poison)
    return out + poison


# --------------------------------------------------------------------------
# reference-named helpers (renderer.py:127-165)
# --------------------------------------------------------------------------
def normalize_points(input_pts, xyz_min, xyz_max):
    """renderer.py:127-128 (torch elementwise; used by callers, not the hot path)."""
    return 2 * (input_pts - xyz_min) / (xyz_max - xyz_min) - 1


def denormalize_points(input_pts, xyz_min, xyz_max):
    """renderer.py:130-131."""
    return (input_pts + 1) / 2 * (xyz_max - xyz_min) + xyz_min


def draw_jitter(n_azi, n_ele):
    """The two CPU-generator draws of renderer.py:149,153 (same order)."""
    u_azi = torch.rand(n_azi)
    torch.rand(n_ele)  # elevation jitter is multiplied by 0 but consumes the stream
    return u_azi


def ray_directions(n_azi, n_ele, random_azi=True, device=None):
    """renderer.py:133-165 on the GPU: returns (dir [R,3], None, None).

    The azimuth jitter is drawn from the CPU default generator exactly as the
    reference does; directions are computed by the `avr_ray_directions`
    kernel.  (The reference also returns the meshgrid angles; no caller uses
    them, so they are returned as None.)
    """
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    u = draw_jitter(n_azi, n_ele)
    if not random_azi:
        u = torch.zeros_like(u)
    p = render_params(dict(n_azi=n_azi, n_ele=n_ele, n_samples=1, far=1, near=0, xyz_min=-1,
                           xyz_max=1, fs=1, speed=1, pathloss=1), 2)
    dirs = torch.empty(n_azi * n_ele + 2, 3, dtype=torch.float32, device=device)
    u_dev = u.to(device, non_blocking=True)
    _lib.call("avr_ray_directions", ctypes_ref(p), _ptr(u_dev), _ptr(dirs), _stream(device))
    return dirs, None, None


# --------------------------------------------------------------------------
# the drop-in module
# --------------------------------------------------------------------------
class AVRRender(nn.Module):
    """Audio signal rendering (renderer.py:13-124), MI355X-native."""

    def __init__(self, networks_fn, **kwargs) -> None:
        super().__init__()
        self.network_fn = networks_fn
        for k in _RENDER_KEYS:
            setattr(self, k, kwargs[k])
        self._cfg = {k: kwargs[k] for k in _RENDER_KEYS}
        self.ray_range = None  # (r0, r1) when rays are sharded over GPUs
        # fold the signal network's last layer into the render when the
        # network offers it (avr_amd.model networks; FusedHeadCore)
        self.fused_head = bool(kwargs.get("fused_head", True))
        # Non-finite network outputs: the ray reduction never loads a 16-byte
        # chunk whose elements are all masked, so a NaN/Inf confined to masked
        # elements does not reach the spectrum here, whereas the reference's
        # `signal * mask` turns it into NaN (renderer.py:82,89) and its runner
        # then skips the step (avr_runner.py:183-185).  With
        # propagate_nonfinite=True any non-finite attn/signal element poisons
        # the output exactly like the reference (one extra read of the
        # network output, no host synchronisation).
        self.propagate_nonfinite = bool(kwargs.get("propagate_nonfinite", False))
        # 16-bit networks through the fused head: form every signal element
        # on the matrix cores and round it to the network's 16-bit type before
        # the masked ray sum, as the reference's fp16 network output is
        # rounded (renderer_cpu.py:73,80,90; csrc/head_exact.hip).
        # exact_head=False keeps the linear-algebra head of csrc/head.hip,
        # which sums the exact products (about 3e-4 relative off the
        # reference's rounded render at fp16).
        self.exact_head = bool(kwargs.get("exact_head", True))
        # the fused head's backward applies the last hidden layer's ReLU mask
        # when that layer hands it over (False: the layer keeps its own
        # threshold_backward; bitwise the same gradients)
        self.head_relu_link = bool(kwargs.get("head_relu_link", True))
        self._pcache = {}
        self._pcache_lock = threading.Lock()
        # jitter the sampling kernel reads at run time while a HIP graph is
        # captured (avr_amd.graph): a device tensor or a device address
        self._jitter_dev = None
        self._staged = None  # (device address, pose_out) of a staged pose block (avr_amd.graph)
        # bench/tuning instrumentation: an object whose events(...) returns the
        # hipEvent_t pair recorded around the ray reduction (bench.KernelTimer)
        self.kernel_timer = None

    # -- stages, exposed for tests and for callers that bring their own network
    def _device(self, rays_o):
        if rays_o.is_cuda:
            return rays_o.device
        if not torch.cuda.is_available():
            raise RuntimeError("avr_amd.AVRRender needs a HIP device (no CPU fallback)")
        return torch.device("cuda", torch.cuda.current_device())

    def sample(self, rays_o, position_tx, direction_tx=None, u_azi=None):
        """Ray generation + sampling (renderer.py:53-62) -> network inputs.

        Returns (pts, view, tx, dir_tx_or_None, geom) where geom carries the
        device tensors the render core needs.  When `self.ray_range` is set
        (ray sharding, avr_amd.parallel) only rays [r0, r1) are sampled; the
        jitter draw and the full direction set are still computed so every
        shard sees the same sphere.
        """
        if self._staged is not None:
            return self._sample_staged(position_tx.size(0), direction_tx is not None)
        dev = self._device(rays_o)
        B = position_tx.size(0)
        u_dev = self._jitter_dev if u_azi is None else None
        if u_azi is not None and u_azi.is_cuda:
            # jitter already on the device (RCCL broadcast by RayShardedRender):
            # the sampling kernel reads it there, no host round trip
            u_dev, u_azi = u_azi.to(dev, torch.float32).contiguous(), None
        if u_azi is None and u_dev is None:
            u_azi = draw_jitter(self.n_azi, self.n_ele)
        R_all = int(self.n_azi) * int(self.n_ele) + 2
        r0, r1 = self.ray_range if self.ray_range is not None else (0, R_all)
        if not (0 <= r0 < r1 <= R_all):
            raise ValueError(f"ray_range {self.ray_range} outside [0, {R_all})")
        p0 = self._params(2, r1 - r0)
        R, S = r1 - r0, p0.n_samples
        f32 = dict(dtype=torch.float32, device=dev)
        rays_o = _f32_on(rays_o, dev)
        position_tx = _f32_on(position_tx, dev)
        if direction_tx is not None:
            direction_tx = _f32_on(direction_tx, dev)
        st = _stream(dev)
        pref = ctypes_ref(p0)
        pts = torch.empty(B, R * S, 3, **f32)
        view = torch.empty(B, R * S, 3, **f32)
        tx = torch.empty(B, R * S, 3, **f32)
        dtx = torch.empty(B, R * S, 3, **f32) if direction_tx is not None else None
        with _on(dev):
            if u_dev is not None:
                # graph capture: the jitter is read from device memory at replay
                dirs = torch.empty(R, 3, **f32)
                # (a device tensor, or the device address of a pinned host
                # buffer the captured kernel reads at replay: avr_amd.graph)
                u_ptr = u_dev if isinstance(u_dev, int) else _ptr(u_dev)
                _lib.call("avr_sample_rays_dev", pref, B, u_ptr, r0, _ptr(rays_o),
                          _ptr(position_tx), _ptr(direction_tx), _ptr(dirs), _ptr(pts), _ptr(view),
                          _ptr(tx), _ptr(dtx), st)
            elif p0.n_azi <= _lib.MAX_AZI:
                # one fused launch; the jitter travels in the kernel arguments
                u_host = u_azi.detach()
                if u_host.device.type != "cpu" or u_host.dtype != torch.float32 or not u_host.is_contiguous():
                    u_host = u_host.to("cpu", torch.float32).contiguous()
                dirs = torch.empty(R, 3, **f32)
                _lib.call("avr_sample_rays", pref, B, u_host.data_ptr(), r0, _ptr(rays_o),
                          _ptr(position_tx), _ptr(direction_tx), _ptr(dirs), _ptr(pts), _ptr(view),
                          _ptr(tx), _ptr(dtx), st)
            else:
                dirs_all = torch.empty(R_all, 3, **f32)
                u_dev = u_azi.to(dev, torch.float32)
                d_vals = torch.empty(S, **f32)
                _lib.call("avr_ray_directions", pref, _ptr(u_dev), _ptr(dirs_all), st)
                _lib.call("avr_depth_samples", pref, _ptr(d_vals), st)
                dirs = dirs_all[r0:r1]
                _lib.call("avr_sample_points", pref, B, _ptr(rays_o), _ptr(position_tx),
                          _ptr(direction_tx), _ptr(dirs), _ptr(d_vals), _ptr(pts), _ptr(view),
                          _ptr(tx), _ptr(dtx), st)
        geom = dict(rays_o=rays_o, position_tx=position_tx, dirs=dirs, device=dev, B=B,
                    n_rays=R)
        return pts, view, tx, dtx, geom

    def _sample_staged(self, B, has_dtx):
        """sample() with the pose and the jitter read at run time from the
        staged block `self._staged = (device address, pose_out)` (HIP-graph
        capture with host-side poses, avr_amd.graph): the kernel publishes
        the pose into pose_out [9B] on the device for the render core."""
        staged_ptr, pose_out = self._staged
        dev = pose_out.device
        R_all = int(self.n_azi) * int(self.n_ele) + 2
        r0, r1 = self.ray_range if self.ray_range is not None else (0, R_all)
        p0 = self._params(2, r1 - r0)
        R, S = r1 - r0, p0.n_samples
        f32 = dict(dtype=torch.float32, device=dev)
        pts = torch.empty(B, R * S, 3, **f32)
        view = torch.empty(B, R * S, 3, **f32)
        tx = torch.empty(B, R * S, 3, **f32)
        dtx = torch.empty(B, R * S, 3, **f32) if has_dtx else None
        dirs = torch.empty(R, 3, **f32)
        with _on(dev):
            _lib.call("avr_sample_rays_staged", ctypes_ref(p0), B, staged_ptr, int(has_dtx), r0,
                      _ptr(pose_out), _ptr(dirs), _ptr(pts), _ptr(view), _ptr(tx), _ptr(dtx), _stream(dev))
        geom = dict(rays_o=pose_out[:3 * B].view(B, 3), position_tx=pose_out[3 * B:6 * B].view(B, 3),
                    dirs=dirs, device=dev, B=B, n_rays=R)
        return pts, view, tx, dtx, geom

    def _params(self, T, R):
        """render_params for (T, rays), cached: the scalars never change."""
        key = (T, R)
        p = self._pcache.get(key)
        if p is None:
            with self._pcache_lock:  # nn.DataParallel threads share the module
                p = self._pcache.get(key)
                if p is None:
                    p = render_params(self._cfg, T, n_rays=R)
                    self._pcache[key] = p
        return p

    def render_from_network_output(self, attn, signal, geom, ir_out=None):
        """Render core (renderer.py:74-124) on given network outputs; the IR
        (utils/criterion.py:71) is also written into `ir_out` when given."""
        dev, B = geom["device"], geom["B"]
        S = int(self.n_samples)
        native = (torch.float32, torch.float16, torch.bfloat16)
        if attn.dtype not in native:
            attn = attn.float()
        if signal.dtype not in native:
            signal = signal.float()
        if attn.device != dev:
            attn = attn.to(dev)
        attn = attn.reshape(B, -1)
        if not attn.is_contiguous():
            attn = attn.contiguous()
        T = signal.size(-1)
        if signal.device != dev:
            signal = signal.to(dev)
        signal = signal.reshape(B, -1, T)
        if not signal.is_contiguous():
            signal = signal.contiguous()
        R = geom["n_rays"]
        if attn.size(1) != R * S or signal.size(1) != R * S:
            raise ValueError(f"network output has {signal.size(1)} ray-samples, expected "
                             f"{R}x{S}={R * S}")
        p = self._params(T, R)
        with _on(dev):
            tables = get_tables(p, dev)
            check_config(p, tables)
            if not (torch.is_grad_enabled() and (attn.requires_grad or signal.requires_grad)):
                # inference: the same native call without the autograd node
                out = _render_core_fwd(attn, signal, p, tables, geom["rays_o"],
                                       geom["position_tx"], geom["dirs"], ir_out, self.kernel_timer)[0]
            else:
                out = RenderCore.apply(attn, signal, p, tables, geom["rays_o"], geom["position_tx"],
                                       geom["dirs"], ir_out, self.kernel_timer)
            if self.propagate_nonfinite:
                out = _poison_nonfinite(out, (attn, signal), ir_out)
            return out

    def _head_supported(self, geom, h, weight, dtype):
        """Whether the fused-head kernels take this shape (T <= 4096, <= 4096
        rays per shard, the LDS budget, fp32/bf16/fp16); otherwise the network
        applies its last layer and the plain path renders."""
        if dtype not in (torch.float32, torch.bfloat16, torch.float16):
            return False
        p = self._params(weight.size(0), geom["n_rays"])
        code = {torch.bfloat16: DTYPE_BF16, torch.float16: DTYPE_F16}.get(dtype, DTYPE_F32)
        n = ctypes.c_int32(0)
        lib = _lib.load()
        if lib.avr_head_splits(ctypes_ref(p), geom["B"], h.size(-1), code, ctypes.byref(n)) != 0:
            return False
        if self._exact_for(dtype, h.size(-1)):
            nb = ctypes.c_int64(0)
            return lib.avr_head_exact_layout(ctypes_ref(p), geom["B"], h.size(-1), code, ctypes.byref(n),
                                             ctypes.byref(nb)) == 0
        return True

    def _exact_for(self, dtype, K):
        """The output-rounding-exact head runs for 16-bit networks (csrc/head_exact.hip)."""
        return self.exact_head and dtype in (torch.float16, torch.bfloat16) and K % 16 == 0 and K <= 512

    def render_from_hidden(self, attn, h, weight, dtype, geom, relu_link=None):
        """Render core with the signal head fused (FusedHeadCore): `h` is the
        signal network's last hidden activation [B, R*S, K], `weight` its
        last layer's weight [T, K] (signal = h @ weight^T).  `relu_link`
        (the network's, see model.MLP.hidden): h is a ReLU output the head
        alone consumes; the head's backward then applies that ReLU's mask
        and the link tells the layer to skip its own."""
        dev, B = geom["device"], geom["B"]
        S = int(self.n_samples)
        attn = attn.to(dev).reshape(B, -1)
        if attn.dtype not in (torch.float32, torch.float16, torch.bfloat16):
            attn = attn.float()
        attn = attn.contiguous()
        K, T = h.size(-1), weight.size(0)
        h = h.to(dev, dtype).reshape(B, -1, K).contiguous()
        R = geom["n_rays"]
        if attn.size(1) != R * S or h.size(1) != R * S:
            raise ValueError(f"network output has {h.size(1)} ray-samples, expected {R}x{S}={R * S}")
        p = self._params(T, R)
        with _on(dev):
            tables = get_tables(p, dev)
            check_config(p, tables)
            exact = self._exact_for(dtype, K)
            relu_h = relu_link is not None and torch.is_grad_enabled()
            out = FusedHeadCore.apply(attn, h, weight, dtype, p, tables, geom["rays_o"],
                                      geom["position_tx"], geom["dirs"], not torch.is_grad_enabled(), exact,
                                      relu_h, self.kernel_timer)
            if relu_h:
                relu_link[0] = True
            if self.propagate_nonfinite:
                # the head kernels skip rays with an empty window, so a
                # non-finite h / attn of a masked ray never reaches `out`
                # (the reference's signal = h W^T carries it through its masks)
                out = _poison_nonfinite(out, (attn, h, weight))
            return out

    def forward(self, rays_o, position_tx, direction_tx=None, ch_idx=None):
        """Render [B, F, 2] (real, imag) spectra; see renderer.py:31-124."""
        return self._render(rays_o, position_tx, direction_tx, ch_idx, None)

    def render_ir(self, rays_o, position_tx, direction_tx=None, ch_idx=None):
        """(spectrum [B, F, 2], IR [B, 2(F-1)]): forward plus
        `torch.real(torch.fft.irfft(...))` (utils/criterion.py:71).  Without
        autograd the IR is computed in the same native call; with autograd
        recording it is spectrum_to_ir(out), which differentiates."""
        ir = []
        # the IR inside the render's native call is a forward-only side
        # output; with autograd recording, take it differentiably instead
        grad = torch.is_grad_enabled()
        out = self._render(rays_o, position_tx, direction_tx, ch_idx, None if grad else ir)
        return out, (ir[0] if ir else spectrum_to_ir(out))

    def _render(self, rays_o, position_tx, direction_tx, ch_idx, ir_slot, u_azi=None):
        """Sampling -> network -> render core; `u_azi` (the azimuth jitter,
        host or device) replaces the CPU draw, as RayShardedRender passes
        rank 0's broadcast draw so every ray shard sees one sphere."""
        pts, view, tx, dtx, geom = self.sample(rays_o, position_tx, direction_tx, u_azi=u_azi)
        kw = {} if ch_idx is None else {"ch_idx": ch_idx}
        if getattr(self.network_fn, "accepts_ray_layout", False):
            # our own networks: tell them which inputs repeat over samples /
            # rays so they encode each distinct row once (same values)
            kw["ray_layout"] = (geom["B"], geom["n_rays"], int(self.n_samples))
        net_in = (pts, view, tx) if dtx is None else (pts, view, tx, dtx)
        if self.fused_head and getattr(self.network_fn, "supports_fused_head", False):
            attn, h, weight, dtype = self.network_fn.forward_fused(*net_in, **kw)
            if self._head_supported(geom, h, weight, dtype):
                # our own networks leave the link of h's ReLU (model.MLP.hidden)
                link = getattr(self.network_fn, "_relu_link", None) if self.head_relu_link else None
                self.network_fn.__dict__.pop("_relu_link", None)
                return self.render_from_hidden(attn, h, weight, dtype, geom, link)
            signal = self.network_fn.finish_signal(h)
            return self.render_from_network_output(attn, signal, geom)
        if dtx is not None:
            attn, signal = self.network_fn(pts, view, tx, dtx, **kw)
        else:
            attn, signal = self.network_fn(pts, view, tx, **kw)
        ir_out = None
        if ir_slot is not None:
            F = signal.size(-1) // 2 + 1
            if F >= 2:
                ir_out = torch.empty(geom["B"], 2 * (F - 1), dtype=torch.float32,
                                     device=geom["device"])
                ir_slot.append(ir_out)
        return self.render_from_network_output(attn, signal, geom, ir_out)


# --------------------------------------------------------------------------
# a13: IR synthesis (utils/criterion.py:71 applied to the rendered spectrum)
# --------------------------------------------------------------------------
class _IRFFT(torch.autograd.Function):
    """HIP irfft (avr_irfft) with its adjoint (avr_irfft_bwd) as backward."""

    @staticmethod
    def forward(ctx, out):
        dev = out.device
        B, F = out.size(0), out.size(1)
        n = 2 * (F - 1)
        tw = _ir_twiddle(n, dev)
        ir = torch.empty(B, n, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            _lib.call("avr_irfft", B, F, _ptr(out), _ptr(tw), _ptr(ir), _stream(dev))
        return ir

    @staticmethod
    def backward(ctx, g):
        dev = g.device
        g = g.float().contiguous()
        B, n = g.size(0), g.size(1)
        F = n // 2 + 1
        grad = torch.empty(B, F, 2, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            _lib.call("avr_irfft_bwd", B, F, _ptr(g), _ptr(_ir_twiddle(n, dev)), _ptr(grad), _stream(dev))
        return grad


def spectrum_to_ir(out):
    """[B, F, 2] spectrum -> [B, 2(F-1)] IR with the HIP irfft kernel.

    Same result as `torch.real(torch.fft.irfft(out[...,0] + 1j*out[...,1]))`
    (avr_runner.py:178 + utils/criterion.py:71), and differentiable like it:
    the backward is the adjoint irfft kernel (torch's c2r backward: interior
    bins doubled, no imaginary gradient at DC / Nyquist), so a loss taken on
    the IR (utils/criterion.py:71-98) reaches the render.
    """
    if not out.is_cuda:
        raise RuntimeError("spectrum_to_ir needs a HIP tensor (no CPU fallback)")
    if out.dtype != torch.float32:
        out = out.float()
    return _IRFFT.apply(out.contiguous())


_IRTW: dict = {}


def _ir_twiddle(n, dev):
    key = (dev.index, n)
    tw = _IRTW.get(key)
    if tw is None:
        with _TABLE_LOCK:
            tw = _IRTW.get(key)
            if tw is None:
                tw = torch.empty(n, 2, dtype=torch.float32, device=dev)
                with torch.cuda.device(dev):
                    _lib.call("avr_ir_twiddle", n, _ptr(tw), _stream(dev))
                    # other host threads read it on their own streams
                    torch.cuda.current_stream(dev).synchronize()
                _IRTW[key] = tw
    return tw
