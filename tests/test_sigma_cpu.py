"""CPU checks of the fused sigma networks' host side (`avr_amd/sigma.py`).

The packed weight fragments are run through a software model of the kernel
(`csrc/sigma.hip`): v_mfma_f32_32x32x16_bf16 with the gfx950 operand and
accumulator lane maps (cdna_hip_programming.md §3), the accumulator-as-next-
B-operand chaining, the tile stores and the attn lane.  The model must
reproduce `reference_fwd` (plain PyTorch statement of the unfused bf16
path), which pins the fragment permutation, the chunk layout and the
first-layer input chunking without a GPU.
"""
import numpy as np
import pytest
import torch

from avr_amd import sigma

BF = torch.bfloat16


def mfma(afrag, bfrag, c):
    """One 32x32x16 bf16 MFMA on lane-major fragments: afrag/bfrag [64, 8],
    c [64, 16] fp32 -> c + A B in the C/D lane map."""
    A = torch.zeros(32, 16)
    B = torch.zeros(16, 32)
    for lane in range(64):
        r, h = lane & 31, lane >> 5
        A[r, 8 * h:8 * h + 8] = afrag[lane].float()
        B[8 * h:8 * h + 8, r] = bfrag[lane].float()
    D = A @ B
    out = c.clone()
    lanes = torch.arange(64)
    for i in range(16):
        rows = (i & 3) + 8 * (i >> 2) + 4 * (lanes >> 5)
        out[:, i] += D[rows, lanes & 31]
    return out


def run_model(variant, packed, inputs, extras, slope, bias=None, bias_div=1):
    """Software model of one wave (32 samples, NT = 1) of the kernel."""
    sched = sigma.SCHEDULE[variant]
    chunks = packed.view(-1, sigma.CHUNK // 2)
    lanes = torch.arange(64)
    n = lanes & 31
    h = lanes >> 5
    ks0 = sched[0][1] // 16 + (1 if sched[0][1] % 16 else 0)
    x = []
    for ks in range(ks0):
        f = torch.zeros(64, 8, dtype=BF)
        for lane in range(64):
            c = 2 * ks + int(h[lane])
            src = None
            if c < 5:
                t, div, col = inputs[0][0], inputs[0][1], 8 * c
                src = t[int(n[lane]) // div, col:col + 8]
            elif len(inputs) > 1 and c < 10:
                t, div, col = inputs[1][0], inputs[1][1], 8 * (c - 5)
                src = t[int(n[lane]) // div, col:col + 8]
            if src is not None:
                f[lane] = src.to(BF)
        x.append(f)
    ci = 0
    base_cols = {}
    attn = None
    n_enc = 4
    h1_layer = 8 if variant == sigma.MESHRIR_H1 else -1
    xs = None
    h1 = torch.zeros(32, 512)
    # the chunks in the kernel's stream order (MESHRIR_H1: the signal layer
    # right after the encoder)
    for li in sigma.STREAM_ORDER.get(variant, range(len(sched))):
        M, K, first, co = sched[li]
        OT, KS = -(-M // 32), -(-K // 16)
        inp = xs if li == h1_layer else x
        assert len(inp) == KS
        acc = [torch.zeros(64, 16) for _ in range(OT)]
        for c in range(OT // co):
            fr = chunks[ci][:co * KS * 512].view(co, KS, 64, 8)
            ci += 1
            for o in range(co):
                for ks in range(KS):
                    acc[c * co + o] = mfma(fr[o, ks], inp[ks], acc[c * co + o])
        if li == h1_layer:  # relu(acc + bias) -> h1
            for ot in range(OT):
                for i in range(16):
                    col = 32 * ot + (i & 3) + 8 * (i >> 2) + 4 * h
                    for lane in range(64):
                        r = int(n[lane])
                        h1[r, int(col[lane])] = acc[ot][lane, i] + bias[r // bias_div, int(col[lane])]
            continue
        if li == n_enc - 1 and variant == sigma.MESHRIR_H1:
            xs = []
            for ot in range(OT):
                for s_ in range(2):
                    xs.append(acc[ot][:, 8 * s_:8 * s_ + 8].to(BF))
        if li == n_enc - 1:  # encoder output -> base columns
            for ot in range(OT):
                v = acc[ot]
                if variant == sigma.RAF:
                    v = torch.relu(v)
                for i in range(16):
                    col = 32 * ot + (i & 3) + 8 * (i >> 2) + 4 * h
                    for lane in range(64):
                        base_cols[(int(n[lane]), int(col[lane]))] = v[lane, i].to(BF)
        if OT == 1:
            y = acc[0][:32, 0].to(BF).float()
            attn = torch.abs(torch.where(y > 0, y, y * float(np.float32(slope))).to(BF))
        else:
            x = []
            for ot in range(OT):
                for s in range(2):
                    x.append(torch.relu(acc[ot][:, 8 * s:8 * s + 8]).to(BF))
    if variant == sigma.MESHRIR_H1:
        assert ci == len(chunks)
        return attn, torch.relu(h1).to(BF)
    out_w = 256 if variant == sigma.RAF else 128
    feat = torch.zeros(32, out_w, dtype=BF)
    for (i, c), v in base_cols.items():
        feat[i, c] = v
    idx = torch.arange(32)
    base = torch.cat([feat] + [t[idx // d].to(BF) for t, d in extras], -1)
    assert ci == len(chunks)
    return attn, base


def _weights(variant, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(M, K, generator=g) / np.sqrt(K) for M, K, _, _ in sigma.SCHEDULE[variant]]


def test_fragment_index_covers_every_weight_once():
    for M, K, first in [(128, 40, True), (128, 128, False), (256, 128, False), (1, 128, False),
                        (128, 80, True)]:
        o, k, valid = sigma.fragment_index(M, K, first)
        pairs = set(zip(o[valid].tolist(), k[valid].tolist()))
        assert len(pairs) == M * K == int(valid.sum())


def test_packed_size_matches_library_contract():
    for v in (sigma.MESHRIR, sigma.RAF):
        p = sigma.pack_layers(v, _weights(v, 0))
        assert p.dtype == BF and p.numel() * 2 == 8 * sigma.CHUNK


@pytest.mark.parametrize("variant", [sigma.MESHRIR, sigma.RAF])
def test_kernel_model_matches_reference(variant):
    g = torch.Generator().manual_seed(3)
    ws = _weights(variant, 1)
    packed = sigma.pack_layers(variant, ws)
    S = 8  # rows per ray in the broadcast sources
    if variant == sigma.MESHRIR:
        inputs = [(torch.rand(32, 40, generator=g).half(), 1)]
        extras = [(torch.rand(32 // S, 40, generator=g).half(), S), (torch.rand(1, 40, generator=g).half(), 32)]
        slope = 0.01
    else:
        inputs = [(torch.rand(32, 40, generator=g), 1), (torch.rand(1, 40, generator=g), 32)]
        extras = [(torch.rand(32 // S, 40, generator=g), S), (torch.rand(1, 40, generator=g), 32),
                  (torch.rand(32, 40, generator=g), 1), (torch.rand(1, 40, generator=g), 32)]
        slope = 0.03
    attn, base = run_model(variant, packed, inputs, extras, slope)
    ra, rb = sigma.reference_fwd(variant, ws, inputs, extras, 32, slope)
    # fp32 accumulation order differs (model: per k-step; reference: one GEMM),
    # so a few bf16 roundings may land on the other side: 2 bf16 ulps
    assert base.shape == rb.shape
    torch.testing.assert_close(base.float(), rb.float(), rtol=2 ** -7, atol=1e-3)
    torch.testing.assert_close(attn.float(), ra.float(), rtol=2 ** -7, atol=1e-3)


def test_variant_detection():
    from avr_amd.model import AVRModel, AVRModel_complex
    from avr_amd.workloads import MESHRIR_MODEL, RAF_MODEL

    m = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254), mlp_dtype=torch.bfloat16)
    assert sigma.variant_of(m) == sigma.MESHRIR
    m32 = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254), mlp_dtype=torch.float32)
    assert sigma.variant_of(m32) is None
    r = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=254), mlp_dtype=torch.bfloat16)
    assert sigma.variant_of(r) == sigma.RAF
    # fp16 (tcnn's MLP precision) takes the fused kernel too
    m16 = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254), mlp_dtype=torch.float16)
    assert sigma.variant_of(m16) == sigma.MESHRIR and sigma.h1_ok(m16)
    r16 = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=254), mlp_dtype=torch.float16)
    assert sigma.variant_of(r16) == sigma.RAF
    assert sigma.pack_layers(sigma.RAF, _weights(sigma.RAF, 0), torch.float16).dtype == torch.float16


def test_desc_struct_matches_library():
    import ctypes

    from avr_amd import _lib

    lib = _lib.load()
    assert lib.avr_sigma_desc_size() == ctypes.sizeof(sigma.SigmaDesc)
    b = ctypes.c_int64(0)
    _lib.call("avr_sigma_pack_bytes", sigma.MESHRIR, ctypes.byref(b))
    assert b.value == 8 * sigma.CHUNK


def test_kernel_model_h1_matches_reference():
    """MESHRIR_H1: sigma networks + the signal network's first layer on the
    raw sigma_feat fragments (12 chunks), bias per group."""
    g = torch.Generator().manual_seed(4)
    ws = _weights(sigma.MESHRIR_H1, 2)
    packed = sigma.pack_layers(sigma.MESHRIR_H1, ws)
    assert packed.numel() * 2 == 12 * sigma.CHUNK
    inputs = [(torch.rand(32, 40, generator=g).half(), 1)]
    bias = torch.randn(4, 512, generator=g) * 0.1
    attn, h1 = run_model(sigma.MESHRIR_H1, packed, inputs, [], 0.01, bias=bias, bias_div=8)
    ra, rh = sigma.reference_fwd(sigma.MESHRIR_H1, ws, inputs, [], 32, 0.01, bias=bias, bias_div=8)
    torch.testing.assert_close(h1.float(), rh.float(), rtol=2 ** -7, atol=2e-3)
    torch.testing.assert_close(attn.float(), ra.float(), rtol=2 ** -7, atol=1e-3)
