"""Fused sigma networks for inference (`csrc/sigma.hip`, `avr_sigma_fwd`).

The sigma encoder and decoder of the reference networks are width-128
bias-free ReLU MLPs that tcnn runs as FullyFusedMLP (model.py:117-121,
146-150, 267-277).  With no autograd graph to record, `AVRModel` and
`AVRModel_complex` run them, and the concatenation of the signal network's
input (model.py:221, 325), as one HIP launch: activations stay in registers
from layer to layer (bf16 MFMA, fp32 accumulation) and the only HBM traffic
is the encodings in and `base` + `attn` out.

Weights are packed once per parameter version into MFMA A-operand fragments
(`pack_layers`): fragment (tile ot, k-step ks) holds, for lane l (r = l & 31,
h = l >> 5) and element j, W[32 ot + r][k] with
    k = 16 ks + 8 h + j                      first layer (inputs loaded from memory)
    k = 16 ks + 8 (j >> 2) + 4 h + (j & 3)   later layers (inputs = the previous
                                             layer's accumulator registers)
grouped into 32 KB chunks (one LDS stage each) of CO tiles.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .wcache import cache_lookup, cache_store, capturing

MESHRIR = 0  # AVR_SIGMA_MESHRIR
RAF = 1      # AVR_SIGMA_RAF
MESHRIR_H1 = 2  # AVR_SIGMA_MESHRIR_H1: MESHRIR + the signal network's first layer
MAX_EXTRA = 4
CHUNK = 32768

# per variant: (M, K, first, tiles per chunk) of every layer, in chunk order
SCHEDULE = {
    MESHRIR: [(128, 40, True, 4)] + [(128, 128, False, 4)] * 6 + [(1, 128, False, 1)],
    RAF: [(128, 80, True, 4), (128, 128, False, 4), (128, 128, False, 4), (256, 128, False, 4),
          (128, 256, False, 2), (1, 128, False, 1)],
}
SCHEDULE[MESHRIR_H1] = SCHEDULE[MESHRIR] + [(512, 128, False, 4)]
# the order the kernel streams the layers in, where it is not SCHEDULE's:
# MESHRIR_H1 runs the signal layer (8) right after the encoder (0-3), then
# the decoder (4-7) on the rectified features (csrc/sigma.hip)
STREAM_ORDER = {MESHRIR_H1: [0, 1, 2, 3, 8, 4, 5, 6, 7]}


class FeatSrc(ctypes.Structure):
    """Mirror of `avr_feat_src` (include/avr_hip.h)."""

    _fields_ = [("data", ctypes.c_void_p), ("dtype", ctypes.c_int32), ("rows_div", ctypes.c_int32),
                ("lm_rows", ctypes.c_int64)]


class SigmaDesc(ctypes.Structure):
    """Mirror of `avr_sigma_desc` (include/avr_hip.h)."""

    _fields_ = [("variant", ctypes.c_int32), ("tile_cfg", ctypes.c_int32),
                ("n_samples", ctypes.c_int64), ("leaky_slope", ctypes.c_float),
                ("input", FeatSrc * 2), ("n_extra", ctypes.c_int32),
                ("extra", FeatSrc * MAX_EXTRA), ("extra_width", ctypes.c_int32 * MAX_EXTRA),
                ("bias", ctypes.c_void_p), ("bias_div", ctypes.c_int32), ("dtype", ctypes.c_int32)]


def fragment_index(M, K, first):
    """(o, k, valid) arrays of shape [OT, KS, 64, 8]: the weight element each
    fragment slot holds (see the module docstring)."""
    OT, KS = -(-M // 32), -(-K // 16)
    ot, ks, lane, j = np.meshgrid(np.arange(OT), np.arange(KS), np.arange(64), np.arange(8),
                                  indexing="ij")
    r, h = lane & 31, lane >> 5
    o = 32 * ot + r
    if first:
        k = 16 * ks + 8 * h + j
    else:
        k = 16 * ks + 8 * (j >> 2) + 4 * h + (j & 3)
    valid = (o < M) & (k < K)
    return o, k, valid


_INDEX: dict = {}


def _gather_index(M, K, first, device):
    """Device (row, col) gather indices of fragment_index, invalid slots
    pointing at the zero corner; kept per shape and device, so repacking
    (every optimizer step, or inside a captured HIP graph) does no host copy."""
    key = (M, K, first, device)
    v = _INDEX.get(key)
    if v is None:
        o, k, valid = fragment_index(M, K, first)
        OT, KS = o.shape[:2]
        v = (torch.from_numpy(np.where(valid, o, OT * 32)).to(device),
             torch.from_numpy(np.where(valid, k, KS * 16)).to(device))
        if device.type == "cuda":
            torch.cuda.current_stream(device).synchronize()  # shared across streams
        _INDEX[key] = v
    return v


def pack_layers(variant, weights, dtype=torch.bfloat16):
    """Weights (fp32 [M, K] tensors, in SCHEDULE order) -> packed fragments
    in the MLP dtype (bf16 or fp16), one 32 KB chunk per LDS stage (zero
    padded), as a flat tensor on the weights' device."""
    sched = SCHEDULE[variant]
    if len(weights) != len(sched):
        raise ValueError(f"variant {variant} takes {len(sched)} layers, got {len(weights)}")
    layers = []
    for w, (M, K, first, co) in zip(weights, sched):
        if tuple(w.shape) != (M, K):
            raise ValueError(f"layer shape {tuple(w.shape)} != {(M, K)}")
        oi, ki = _gather_index(M, K, first, w.device)
        OT, KS = oi.shape[:2]
        wp = torch.zeros(OT * 32 + 1, KS * 16 + 1, dtype=torch.float32, device=w.device)
        wp[:M, :K] = w.detach().float()
        frags = wp[oi, ki].to(dtype)  # [OT, KS, 64, 8]
        chunks = []
        for c in range(OT // co):
            part = frags[c * co:(c + 1) * co].reshape(-1)
            pad = CHUNK // 2 - part.numel()
            if pad < 0:
                raise AssertionError("chunk overflow")
            chunks.append(torch.cat([part, part.new_zeros(pad)]))
        layers.append(chunks)
    order = STREAM_ORDER.get(variant, range(len(layers)))
    return torch.cat([c for i in order for c in layers[i]])


def network_layers(mlp):
    """The nn.Linear weights of an `avr_amd.model.MLP`."""
    return [lin.weight for lin in mlp.layers]


def _dims(mlp):
    return [(lin.weight.shape[0], lin.weight.shape[1]) for lin in mlp.layers]


MLP_DTYPES = (torch.bfloat16, torch.float16)


def variant_of(model):
    """AVR_SIGMA_* if the model's sigma networks have exactly the shapes the
    fused kernel implements (and 16-bit MLPs: bf16, or fp16 = tcnn's), else None."""
    enc, dec = model._model_encoder_sigma, model._model_decoder_sigma
    if enc.dtype not in MLP_DTYPES or dec.dtype != enc.dtype:
        return None
    dims = _dims(enc) + _dims(dec)
    for v in (MESHRIR, RAF):
        if dims == [(M, K) for M, K, _, _ in SCHEDULE[v]]:
            return v
    return None


def h1_ok(model):
    """MESHRIR_H1 applies: an AVRModel whose signal network starts with a
    bias-free 208 -> 512 layer on [sigma_feat 128 | dir 40 | tx 40] in the
    sigma networks' 16-bit dtype and has at least one more hidden layer."""
    sig = model._model_signal
    return (variant_of(model) == MESHRIR and sig.dtype == model._model_encoder_sigma.dtype
            and len(sig.layers) >= 3
            and tuple(sig.layers[0].weight.shape) == (512, 208))


class SigmaWeights:
    """Packed fragments of a model's sigma networks, repacked when any weight
    changes (parameter version counters)."""

    def get(self, variant, params, dtype=torch.bfloat16):
        if capturing():  # a captured graph repacks at every replay
            return pack_layers(variant, params, dtype)
        key = (variant, dtype) + tuple((p.data_ptr(), p._version) for p in params)
        hit = cache_lookup(self, "_entry", key)
        if hit is not None:
            return hit
        return cache_store(self, "_entry", key, pack_layers(variant, params, dtype))


def _src(t, rows_div):
    """FeatSrc of a [rows, width] tensor, or of a level-major [L, rows, 2]
    hash-grid output (HashGridEncoding.forward_level_major)."""
    if t.dtype == torch.float16:
        code = _lib.DTYPE_F16
    elif t.dtype == torch.float32:
        code = _lib.DTYPE_F32
    else:
        raise TypeError(f"sigma inputs must be fp16 or fp32, got {t.dtype}")
    if not t.is_contiguous() or t.data_ptr() % 16:
        raise ValueError("sigma inputs must be contiguous and 16-byte aligned")
    lm = int(t.size(1)) if t.dim() == 3 else 0
    return FeatSrc(t.data_ptr(), code, int(rows_div), lm)


def _width(t):
    return int(t.size(0) * t.size(2)) if t.dim() == 3 else int(t.size(1))


def _rows(t, idx):
    """Rows idx of a row-major or level-major source as [len(idx), width]."""
    if t.dim() == 3:
        return t[:, idx].permute(1, 0, 2).reshape(len(idx), -1)
    return t[idx]


def sigma_fwd(variant, packed, n_samples, inputs, extras, out_width, slope, tile_cfg=0, bias=None,
              bias_div=1):
    """One launch: inputs = [(tensor [rows, 40] or level-major [20, rows, 2],
    rows_div)] (1 for MESHRIR, 2 for RAF); extras = [(tensor, rows_div)]
    appended after the MLP output.  The MLP dtype is the packed weights'
    (bf16 or fp16).  Returns (attn [N], base [N, out_width + sum widths]) in it."""
    dev = packed.device
    dtype = packed.dtype
    if dtype not in MLP_DTYPES:
        raise TypeError(f"packed sigma weights must be bf16 or fp16, got {dtype}")
    widths = [_width(t) for t, _ in extras]
    ldb = out_width + sum(widths)
    if ldb % 8:
        raise ValueError("concatenated feature width must be a multiple of 8")
    base = torch.empty(n_samples, ldb, dtype=dtype, device=dev)
    attn = torch.empty(n_samples, dtype=dtype, device=dev)
    d = SigmaDesc()
    d.dtype = _lib.DTYPE_F16 if dtype == torch.float16 else _lib.DTYPE_BF16
    d.variant = variant
    d.tile_cfg = tile_cfg
    d.n_samples = n_samples
    d.leaky_slope = float(np.float32(slope))
    for i, (t, div) in enumerate(inputs):
        if _width(t) != 40:
            raise ValueError("sigma network inputs are 40-wide encodings")
        d.input[i] = _src(t, div)
    d.n_extra = len(extras)
    for i, (t, div) in enumerate(extras):
        d.extra[i] = _src(t, div)
        d.extra_width[i] = widths[i]
    if bias is not None:
        if bias.dtype != torch.float32 or not bias.is_contiguous() or bias.size(-1) != 512:
            raise ValueError("bias must be a contiguous fp32 [groups, 512] tensor")
        d.bias = bias.data_ptr()
        d.bias_div = int(bias_div)
    keep = [t for t, _ in list(inputs) + list(extras)]  # noqa: F841  (alive across the call)
    st = torch.cuda.current_stream(dev).cuda_stream
    _lib.call("avr_sigma_fwd", ctypes.byref(d), ctypes.c_void_p(packed.data_ptr()),
              ctypes.c_void_p(base.data_ptr()), int(ldb), ctypes.c_void_p(attn.data_ptr()),
              ctypes.c_void_p(st))
    return attn, base


def reference_fwd(variant, weights, inputs, extras, n_samples, slope, bias=None, bias_div=1,
                  dtype=torch.bfloat16):
    """Plain PyTorch statement of the same computation with the unfused
    16-bit path's roundings (fp32 GEMMs on `dtype`-rounded operands, `dtype`
    outputs); the test oracle for `sigma_fwd`.  Runs on any device."""
    bf = dtype

    def lin(x, w, relu):
        y = (x.float() @ w.to(bf).float().t())
        if relu:
            y = torch.relu(y)
        return y.to(bf)

    idx = torch.arange(n_samples, device=weights[0].device)
    x = torch.cat([_rows(t, idx // div).to(bf) for t, div in inputs], -1)
    w_h1 = None
    if variant == MESHRIR_H1:
        weights, w_h1 = weights[:-1], weights[-1]
    nw = len(weights)
    n_enc = 4
    for i in range(n_enc - 1):
        x = lin(x, weights[i], True)
    feat = lin(x, weights[n_enc - 1], variant == RAF)
    x = torch.relu(feat)
    for i in range(n_enc, nw - 1):
        x = lin(x, weights[i], True)
    a = lin(x, weights[nw - 1], False).float()
    attn = torch.abs(torch.where(a > 0, a, a * float(np.float32(slope))).to(bf))
    if w_h1 is not None:
        h1 = torch.relu(feat.float() @ w_h1.to(bf).float().t() + bias[idx // bias_div])
        return attn.view(-1), h1.to(bf)
    base = torch.cat([feat] + [_rows(t, idx // div).to(bf) for t, div in extras], -1)
    return attn.view(-1), base
