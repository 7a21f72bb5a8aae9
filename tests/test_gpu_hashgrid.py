"""GPU: hash-grid encoding kernels against oracle/hashgrid_oracle.py.

Parity with tiny-cuda-nn itself is unpinned (tcnn is not vendored in the
reference and cannot be installed offline); these tests pin the HIP kernels
to the repo's restatement of upstream tcnn's GridEncoding algorithm."""
import numpy as np
import pytest
import torch

from avr_amd.options import KernelOptions

from oracle import hashgrid_oracle as hgo

from avr_amd.encoding import HashGridEncoding, level_layout

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CFG = dict(otype="HashGrid", n_levels=20, n_features_per_level=2, log2_hashmap_size=18,
           base_resolution=16)


def _points(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, size=(n, 3)).astype(np.float32)
    x[:8] = np.array([[0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5], [1, 0, 1], [0, 1, 0],
                      [0.999999, 0.0, 0.25], [1e-7, 1 - 1e-7, 0.5], [0.25, 0.75, 1.0]], np.float32)
    return x


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("n", [4096, 20000])  # 20000: the level-major dispatch (>= 16384 points)
def test_forward_matches_restatement(dtype, n):
    """fp32 encodings within 2e-6 of the restatement (same fma chain), fp16
    encodings bit-identical to it (half weight, half fma chain, tcnn's
    kernel_grid with T = half)."""
    enc = HashGridEncoding(3, CFG, dtype=dtype, seed=5).to(DEV)
    with torch.no_grad():
        enc.params.uniform_(-1, 1)
    x = _points(n, 0)
    out = enc(torch.from_numpy(x).to(DEV)).detach().float().cpu().numpy()
    # fp16 encodings read fp16 tables (tcnn's param precision), fp32 ones fp32
    table = enc.params.detach().to(enc.param_dtype).float().cpu().numpy()
    if dtype == torch.float16:
        # tcnn's fp16 GridEncoding: half weights, half fma chain in corner
        # order -- the same half values, bit for bit
        ref = hgo.encode(x, table, enc._off, enc._scale, enc._res, table_dtype=np.float16)
        np.testing.assert_array_equal(out, ref)
    else:
        ref = hgo.encode(x, table, enc._off, enc._scale, enc._res)
        np.testing.assert_allclose(out, ref, rtol=2e-6, atol=2e-6)


BWD_IMPLS = ["partitioned", "atomic"]  # avr_hashgrid_bwd_partitioned (training's) and avr_hashgrid_bwd


@pytest.mark.parametrize("impl", BWD_IMPLS)
def test_backward_matches_restatement(impl, monkeypatch):
    cfg = dict(CFG, n_levels=8, log2_hashmap_size=14)
    enc = HashGridEncoding(3, cfg, dtype=torch.float32, seed=6, options=KernelOptions(hashgrid_bwd=impl)).to(DEV)
    x = _points(2048, 1)
    xt = torch.from_numpy(x).to(DEV)
    out = enc(xt)
    rng = np.random.default_rng(2)
    g = rng.standard_normal(size=out.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).to(DEV))
    ref = hgo.encode_backward(x, g, enc._off, enc._scale, enc._res, enc.n_params)
    got = enc.params.grad.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


def test_level_layout_matches_tcnn_rule():
    off, scale, res = level_layout(20, 18, 16)
    sizes = np.diff(off)
    assert list(res[:4]) == [16, 32, 64, 128]
    assert list(sizes[:4]) == [4096, 32768, 262144, 262144]
    assert int(off[-1]) * 2 == 9510912  # 9.51M params, SURVEY.md §8 a5


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_level_major_forward_is_transposed_forward(dtype):
    """avr_hashgrid_fwd_lm: same values as the row-major kernel, [L, N, 2]."""
    enc = HashGridEncoding(3, CFG, dtype=dtype, seed=7).to(DEV)
    with torch.no_grad():
        enc.params.uniform_(-1, 1)
        for n in (8, 255, 4097, 16384, 20001):
            x = torch.from_numpy(_points(n, 1)).to(DEV)
            a = enc(x)
            b = enc.forward_level_major(x)
            assert b.shape == (20, n, 2)
            assert torch.equal(a, b.permute(1, 0, 2).reshape(n, 40))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_level_major_forward_on_ray_points(dtype):
    """Ray-ordered points (consecutive samples 1.3e-3 apart, as the renderer
    lays them out): the level-major kernel (grouped corner loads for fp16
    tables) equals the per-point kernel bit for bit on every level, the
    coarse ones where neighbouring lanes share cells included."""
    enc = HashGridEncoding(3, CFG, dtype=dtype, seed=8).to(DEV)
    rng = np.random.default_rng(3)
    o = rng.uniform(0.2, 0.8, size=(16, 1, 3))
    d = rng.standard_normal(size=(16, 1, 3))
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    t = np.arange(256)[None, :, None] * 1.3e-3
    x = torch.from_numpy(np.clip(o + d * t, 0, 1).reshape(-1, 3).astype(np.float32)).to(DEV)
    with torch.no_grad():
        enc.params.uniform_(-1, 1)
        a = enc(x)  # 4096 points: the per-point kernel
        b = enc.forward_level_major(x)
        assert torch.equal(a, b.permute(1, 0, 2).reshape(x.size(0), 40))


def _ray_points(n_rays, n_samples, seed, step=1.3e-3):
    """Ray-ordered points as the renderer lays them out: many consecutive
    samples in one coarse cell (atomic contention on the coarse levels)."""
    rng = np.random.default_rng(seed)
    o = rng.uniform(0.2, 0.8, size=(n_rays, 1, 3))
    d = rng.standard_normal(size=(n_rays, 1, 3))
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    t = np.arange(n_samples)[None, :, None] * step
    return np.clip(o + d * t, 0, 1).reshape(-1, 3).astype(np.float32)


@pytest.mark.parametrize("impl", BWD_IMPLS)
@pytest.mark.parametrize("log2", [18, 20])
@pytest.mark.parametrize("gdtype", [torch.float32, torch.float16])
def test_backward_reference_size_tables(log2, gdtype, impl, monkeypatch):
    """The backward where it runs: 20 levels at the reference's table sizes
    (2^18 everywhere, 2^20 for MeshRIR's direction grid,
    config_files/avr_meshrir.yml:56-61), ray-ordered points (equal
    addresses within a wave and across waves: the run-sum and the fp32
    atomics both exercised) plus random ones (hash collisions on the fine
    levels), with fp32 and fp16 upstream gradients (an fp16 encoding's
    grad_out is fp16), against the float64 scatter-add of the restatement.
    fp32 sums in any order: 1e-5 relative to the gradient's scale.  The
    first samples of 300 rays sit on one point (every ray of a pose starts at
    the listener): hundreds of adds into the same entries."""
    cfg = dict(CFG, log2_hashmap_size=log2)
    enc = HashGridEncoding(3, cfg, dtype=gdtype, seed=9, options=KernelOptions(hashgrid_bwd=impl)).to(DEV)
    x = np.concatenate([_ray_points(48, 256, 4), _points(8192, 5), _ray_points(300, 16, 7, step=2e-3)[:1].repeat(300, 0),
                        _points(37, 8)])
    xt = torch.from_numpy(x).to(DEV)
    out = enc(xt)
    assert out.dtype == gdtype
    rng = np.random.default_rng(6)
    g = rng.standard_normal(size=out.shape).astype(np.float32)
    gt = torch.from_numpy(g).to(DEV).to(gdtype)
    out.backward(gt)
    g_used = gt.float().cpu().numpy()  # the values the kernel reads
    ref = hgo.encode_backward(x, g_used, enc._off, enc._scale, enc._res, enc.n_params)
    got = enc.params.grad.double().cpu().numpy()
    scale = np.abs(ref).max()
    assert scale > 0
    err = np.abs(got - ref).max() / scale
    assert err < 1e-5, err
    # every touched entry is touched in both, and no other
    np.testing.assert_array_equal(got != 0, ref != 0)


@pytest.mark.parametrize("n", [1, 3000, 16384, 16897, 40000])
def test_partitioned_backward_accumulates(n):
    """avr_hashgrid_bwd_partitioned adds into grad_params (+=) and equals the
    atomic kernel: one point and 3000 (below 16384 points it runs the atomic
    kernel itself), and the partitioned passes at 16384, a ragged last chunk
    (16897 = 33 x 512 + 1) and 40000 random points."""
    import ctypes

    from avr_amd import _lib
    from avr_amd.encoding import _code

    enc = HashGridEncoding(3, dict(CFG, log2_hashmap_size=16), dtype=torch.float16, seed=10).to(DEV)
    x = torch.from_numpy(_points(max(n, 8), 11)[-n:].copy()).to(DEV)
    L = enc.n_levels
    g = torch.randn(n, 2 * L, device=DEV).half()
    st = torch.cuda.current_stream(DEV).cuda_stream
    meta = (enc._off.ctypes.data, enc._scale.ctypes.data, enc._res.ctypes.data)
    a = torch.zeros(enc.n_params, device=DEV)
    _lib.call("avr_hashgrid_bwd", n, L, x.data_ptr(), g.data_ptr(), _code(g.dtype), *meta, a.data_ptr(), st)
    nb = ctypes.c_int64()
    _lib.call("avr_hashgrid_bwd_workspace", n, L, enc._off.ctypes.data, ctypes.byref(nb))
    ws = torch.empty(nb.value, dtype=torch.uint8, device=DEV)
    base = torch.randn(enc.n_params, device=DEV)
    b = base.clone()
    _lib.call("avr_hashgrid_bwd_partitioned", n, L, x.data_ptr(), g.data_ptr(), _code(g.dtype), *meta,
              b.data_ptr(), ws.data_ptr(), nb.value, st)
    torch.cuda.synchronize()
    scale = float(a.abs().max())
    assert float((b - base - a).abs().max()) <= 1e-5 * scale + 1e-6


@pytest.mark.parametrize("n", [0, 1, 3000, 16897, 40000, 262144])
def test_partitioned_backward_set_overwrites(n):
    """avr_hashgrid_bwd_partitioned_set writes the gradient (=) over a table
    full of garbage (NaN): equal to the += form into zeros wherever a single
    reduce slice owns the partition (bit for bit), within fp32 reassociation
    where several slices add atomically, and zero everywhere nothing
    contributes.  n = 0 clears; below 16384 points the atomic path runs on a
    cleared table; 262,144 points include multi-slice (hot) partitions."""
    import ctypes

    from avr_amd import _lib
    from avr_amd.encoding import _code

    enc = HashGridEncoding(3, dict(CFG, log2_hashmap_size=16), dtype=torch.float16, seed=10).to(DEV)
    m = max(n, 8)
    x = torch.from_numpy(_points(m, 12)[-n:].copy() if n else _points(8, 12)[:0].copy()).to(DEV)
    L = enc.n_levels
    g = torch.randn(n, 2 * L, device=DEV).half()
    st = torch.cuda.current_stream(DEV).cuda_stream
    meta = (enc._off.ctypes.data, enc._scale.ctypes.data, enc._res.ctypes.data)
    nb = ctypes.c_int64()
    _lib.call("avr_hashgrid_bwd_workspace", n, L, enc._off.ctypes.data, ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 256), dtype=torch.uint8, device=DEV)
    a = torch.zeros(enc.n_params, device=DEV)
    _lib.call("avr_hashgrid_bwd_partitioned", n, L, x.data_ptr() if n else a.data_ptr(),
              g.data_ptr() if n else a.data_ptr(), _code(g.dtype), *meta, a.data_ptr(), ws.data_ptr(),
              nb.value, st)
    b = torch.full((enc.n_params,), float("nan"), device=DEV)
    _lib.call("avr_hashgrid_bwd_partitioned_set", n, L, x.data_ptr() if n else a.data_ptr(),
              g.data_ptr() if n else a.data_ptr(), _code(g.dtype), *meta, b.data_ptr(), ws.data_ptr(),
              nb.value, st)
    torch.cuda.synchronize()
    assert torch.isfinite(b).all()
    scale = float(a.abs().max()) if n else 1.0
    assert float((b - a).abs().max()) <= 1e-5 * scale
    assert torch.equal(a == 0, b == 0)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_level_major_unit_map_is_bit_identical(dtype):
    """avr_hashgrid_fwd_lm_unit (the (x + 1) / 2 map applied on load) equals
    mapping first and encoding (model.py:187-189), bit for bit, including
    the end points of [-1, 1]."""
    from avr_amd.model import _unit

    enc = HashGridEncoding(3, CFG, dtype=dtype, seed=13).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(14)
    x = torch.rand(100003, 3, device=DEV, generator=g) * 2 - 1
    x[:3] = torch.tensor([[-1.0, 1.0, 0.0], [1.0, -1.0, -1 + 2 ** -24], [0.5, -0.5, 1 - 2 ** -24]], device=DEV)
    with torch.no_grad():
        a = enc.forward_level_major(x, unit_map=True)
        b = enc.forward_level_major(_unit(x))
    torch.cuda.synchronize()
    assert torch.equal(a, b)
