"""CPU restatement of the hash-grid encoding — TEST INFRASTRUCTURE ONLY.

Parity UNPINNED: the reference calls tinycudann's GridEncoding
(model.py:66-68, 258-263), which is not vendored in /root/reference and is
unavailable offline (requirements.txt:11, unversioned git URL).  This file
restates upstream tiny-cuda-nn's published GridEncoding algorithm (hash
type "CoherentPrime", N-linear interpolation, +0.5 level staggering, dense
levels while res^3 fits the table, the corner sum accumulated in the table
type T as kernel_grid's `result = fma((T)weight, grid_val(...), result)`)
in numpy, and checks the HIP kernel against it; nothing here proves
agreement with tcnn's own numbers.

The backward (encode_backward) sums in float64.  tcnn accumulates an fp16
grid's gradient with half2 atomics (grad_t = T when 2 features per level);
the HIP kernel adds in fp32 instead, a deliberate deviation (more precise,
and tcnn's atomic order is not reproducible anyway): DESIGN.md §9b.
"""
from __future__ import annotations

import numpy as np

PRIMES = (np.uint64(1), np.uint64(2654435761), np.uint64(805459861))


def _index(size, res, g):
    """Dense index while res^3 <= size, coherent-prime hash otherwise; mod size."""
    g = g.astype(np.uint64)
    stride = 1
    idx = np.zeros(g.shape[0], dtype=np.uint64)
    dense_ok = True
    for d in range(3):
        if stride > size:
            dense_ok = False
            break
        idx = (idx + g[:, d] * np.uint64(stride)) & np.uint64(0xFFFFFFFF)
        stride *= res
    if size < stride or not dense_ok:
        h = np.zeros(g.shape[0], dtype=np.uint64)
        for d in range(3):
            h ^= (g[:, d] * PRIMES[d]) & np.uint64(0xFFFFFFFF)
        idx = h
    return (idx % np.uint64(size)).astype(np.int64)


def _hfma(w16, v16, acc16):
    """Correctly rounded half-precision fma (w*v + acc, one rounding): the
    product of two halves and the sum with a half are exact in float64 for
    every case that can change the half result, then one float64 -> float16
    round to nearest even."""
    return (w16.astype(np.float64) * v16.astype(np.float64) + acc16.astype(np.float64)).astype(np.float16)


def encode(x, params, offsets, scales, res, table_dtype=np.float32):
    """x [N,3] float32 in [0,1]; params [n_entries*2] -> [N, 2L] float32.

    table_dtype float32: the fp32 corner chain acc = fma(w, v, acc) (tcnn's
    kernel_grid with T = float).  table_dtype float16 (tcnn's default
    encoding precision, model.py:66-68): the table read as half, the weight
    rounded to half, acc = fma((half)w, v, acc) in half in corner order (x
    bit fastest), the half result returned upcast (exact)."""
    x = np.asarray(x, np.float32)
    half = np.dtype(table_dtype) == np.float16
    table = np.asarray(params, np.float32).reshape(-1, 2)
    if half:
        table = table.astype(np.float16)
    N, L = x.shape[0], len(scales)
    out = np.zeros((N, 2 * L), np.float32)
    for l in range(L):
        size = int(offsets[l + 1] - offsets[l])
        p = (np.float64(scales[l]) * x.astype(np.float64) + 0.5).astype(np.float32)
        cell = np.floor(p)
        frac = (p - cell).astype(np.float32)
        cell = cell.astype(np.int64)
        acc = np.zeros((N, 2), np.float16 if half else np.float32)
        for k in range(8):
            w = np.ones(N, np.float32)
            g = np.empty((N, 3), np.int64)
            for d in range(3):
                if k & (1 << d):
                    w = (w * frac[:, d]).astype(np.float32)
                    g[:, d] = cell[:, d] + 1
                else:
                    w = (w * (np.float32(1) - frac[:, d])).astype(np.float32)
                    g[:, d] = cell[:, d]
            v = table[offsets[l] + _index(size, int(res[l]), g)]
            if half:
                acc = _hfma(w.astype(np.float16)[:, None], v, acc)
            else:
                acc = (w[:, None].astype(np.float64) * v + acc).astype(np.float32)
        out[:, 2 * l: 2 * l + 2] = acc.astype(np.float32)
    return out


def encode_backward(x, grad_out, offsets, scales, res, n_params):
    """Scatter-add of grad_out into the parameter vector (the adjoint of encode)."""
    x = np.asarray(x, np.float32)
    g_out = np.asarray(grad_out, np.float64)
    grad = np.zeros((n_params // 2, 2), np.float64)
    N, L = x.shape[0], len(scales)
    for l in range(L):
        size = int(offsets[l + 1] - offsets[l])
        p = (np.float64(scales[l]) * x.astype(np.float64) + 0.5).astype(np.float32)
        cell = np.floor(p)
        frac = (p - cell).astype(np.float32)
        cell = cell.astype(np.int64)
        for k in range(8):
            w = np.ones(N, np.float32)
            g = np.empty((N, 3), np.int64)
            for d in range(3):
                if k & (1 << d):
                    w = (w * frac[:, d]).astype(np.float32)
                    g[:, d] = cell[:, d] + 1
                else:
                    w = (w * (np.float32(1) - frac[:, d])).astype(np.float32)
                    g[:, d] = cell[:, d]
            e = offsets[l] + _index(size, int(res[l]), g)
            np.add.at(grad, e, w[:, None] * g_out[:, 2 * l: 2 * l + 2])
    return grad.reshape(-1)
