"""GPU: the reference's networks (model.py) on HIP hash grids + PyTorch MLPs,
driven by the drop-in renderer — one training step end to end."""
import pytest
import torch

from avr_amd import AVRRender, spectrum_to_ir
from avr_amd.model import AVRModel, AVRModel_complex
from avr_amd.workloads import MESHRIR_MODEL, RAF_MODEL, WORKLOADS

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _step(model, w, dtx):
    r = AVRRender(model, **w.render).to(DEV)
    opt = torch.optim.Adam(r.parameters(), lr=1e-3)
    g = torch.Generator(device=DEV).manual_seed(0)
    ro = torch.rand(w.batch, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(w.batch, 3, device=DEV, generator=g) * 2 - 1
    out = r(ro, tx, dtx) if dtx is not None else r(ro, tx)
    target = torch.randn_like(out)
    loss = (out - target).abs().mean()
    opt.zero_grad()
    loss.backward()
    grads = {n: p.grad for n, p in r.named_parameters()}
    assert all(v is not None and torch.isfinite(v).all() for v in grads.values())
    assert any(float(v.abs().sum()) > 0 for k, v in grads.items() if "encoding" in k)
    opt.step()
    return out


@pytest.mark.parametrize("mlp_dtype", [torch.float32, torch.bfloat16])
def test_raf_model_training_step(mlp_dtype):
    w = WORKLOADS["c1_meshrir_plumbing"].replace(name="raf_small", **{k: v for k, v in WORKLOADS[
        "c3_raf_furnished_b4"].render.items() if k not in ("n_azi", "n_ele", "n_samples")})
    w = w.replace(T=RAF_MODEL["signal_output_dim"], batch=2)
    model = AVRModel_complex(RAF_MODEL, mlp_dtype=mlp_dtype).to(DEV)
    dtx = torch.nn.functional.normalize(torch.randn(w.batch, 3, device=DEV), dim=-1)
    out = _step(model, w, dtx)
    assert out.shape == (2, RAF_MODEL["signal_output_dim"] // 2 + 1, 2)
    ir = spectrum_to_ir(out.detach())
    assert torch.isfinite(ir).all()


def test_meshrir_model_training_step():
    cfg = dict(MESHRIR_MODEL, signal_output_dim=1022)
    w = WORKLOADS["c1_meshrir_plumbing"].replace(T=1022)  # T large enough that delays fit
    model = AVRModel(cfg).to(DEV)
    out = _step(model, w, None)
    assert out.shape == (1, 512, 2)


@pytest.mark.parametrize("cls", ["AVRModel", "AVRModel_complex"])
def test_ray_layout_grouped_encoding_matches_flat(cls):
    """With ray_layout the per-ray / per-pose inputs are encoded once per group;
    the network output must be bit-identical to the flat call and the
    parameter gradients equal up to fp32 summation order."""
    w = WORKLOADS["c1_meshrir_plumbing"]
    B, R, S = 2, w.n_rays, w.n_samples
    if cls == "AVRModel":
        model = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254)).to(DEV)
    else:
        model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=254)).to(DEV)
    r = AVRRender(model, **w.render)
    g = torch.Generator(device=DEV).manual_seed(3)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
    torch.manual_seed(0)
    pts, view, txs, dts, geom = r.sample(ro, tx, dtx if cls != "AVRModel" else None)
    args = (pts, view, txs) if cls == "AVRModel" else (pts, view, txs, dts)
    outs, grads = [], []
    for layout in (None, (B, R, S)):
        model.zero_grad(set_to_none=True)
        attn, sig = model(*args, ray_layout=layout)
        (attn.float().sum() + (sig.float() * 1e-2).sum()).backward()
        outs.append((attn.detach(), sig.detach()))
        grads.append({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert grads[0].keys() == grads[1].keys()
    # fp16 feature grids (AVRModel): the group's summed gradient is rounded
    # to fp16 once (the flat path adds the fp16 row gradients in fp32)
    rtol = 2e-4 if cls == "AVRModel_complex" else 2e-3
    for n in grads[0]:
        a, b = grads[1][n], grads[0][n]
        err = float((a - b).norm() / b.norm().clamp_min(1e-30))
        assert err < rtol, (n, err)


@pytest.mark.parametrize("N,M,K", [(83200, 512, 512), (83200, 1600, 512), (5003, 512, 336),
                                   (300, 128, 80), (33, 8, 16), (147712, 256, 128), (147712, 512, 416),
                                   (77, 136, 24)])
def test_linear_wgrad_kernel_matches_fp32(N, M, K):
    """avr_linear_wgrad (split-K bf16 MFMA) against an fp32 GEMM of the same
    bf16 operands (products are exact in fp32; only the summation order
    differs)."""
    from avr_amd.model import _hip_wgrad_ok, _wgrad_hip

    g = torch.Generator(device=DEV).manual_seed(N + M + K)
    gy = torch.randn(N, M, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(N, K, device=DEV, generator=g).to(torch.bfloat16)
    assert _hip_wgrad_ok(gy, x)
    out = _wgrad_hip(gy, x)
    ref = gy.double().t() @ x.double()
    err = float((out.double() - ref).norm() / ref.norm())
    assert err < 5e-5, err
    # deterministic
    assert torch.equal(out, _wgrad_hip(gy, x))


def test_linear_wgrad_exact_on_small_integers():
    """Small-integer operands: every partial sum is an integer below 2^24, so
    the fp32 result is exact whatever the order; equal to the int64 GEMM."""
    from avr_amd.model import _wgrad_hip

    g = torch.Generator(device=DEV).manual_seed(5)
    N, M, K = 20011, 264, 200
    gy = torch.randint(-3, 4, (N, M), device=DEV, generator=g)
    x = torch.randint(-3, 4, (N, K), device=DEV, generator=g)
    out = _wgrad_hip(gy.to(torch.bfloat16), x.to(torch.bfloat16))
    ref = (gy.t().double() @ x.double()).to(torch.int64)
    assert torch.equal(out.to(torch.int64), ref)


@pytest.mark.parametrize("M", [1, 3])
def test_wgrad_narrow_output_layer(M):
    """_wgrad of a layer with fewer than 8 outputs (sigma decoder's last):
    zero-padded onto the HIP kernel, against an fp64 GEMM."""
    from avr_amd.model import _wgrad

    g = torch.Generator(device=DEV).manual_seed(M)
    gy = torch.randn(83200, M, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(83200, 256, device=DEV, generator=g).to(torch.bfloat16)
    out = _wgrad(gy, x)
    assert out.shape == (M, 256) and out.dtype == torch.float32 and out.is_contiguous()
    ref = gy.double().t() @ x.double()
    err = float((out.double() - ref).norm() / ref.norm())
    assert err < 5e-5, err


def test_one_output_layer_dgrad_is_the_gemm():
    """_Linear's data gradient for a 1-output layer (broadcast multiply)
    equals the K = 1 GEMM it replaces, bit for bit, in bf16 and fp32."""
    g = torch.Generator(device=DEV).manual_seed(5)
    for dt in (torch.bfloat16, torch.float32):
        gy = torch.randn(83200, 1, device=DEV, generator=g).to(dt)
        w = torch.randn(1, 256, device=DEV, generator=g).to(dt)
        assert torch.equal(gy * w, gy @ w)


@pytest.mark.parametrize("workload", ["c2_meshrir_1024x256x512", "c5_simu_4096x512x2048"])
@pytest.mark.parametrize("enc_dtype", [torch.float16, torch.float32])
def test_ray_pose_bias_kernel_matches_torch_ops(enc_dtype, workload):
    """avr_ray_pose_bias against the torch ops it replaces in the fused
    inference trunk: per-ray / per-pose selection, (x + 1) / 2, the dir and tx
    grids, fp16 -> bf16 -> fp32 rounding, two skinny fp32 GEMMs and their sum
    (only the GEMMs' fp32 summation order differs).  Config 2 (1024 rays per
    pose) takes the one-pose-per-workgroup kernel, config 5 (4094 rays, not a
    multiple of 8) the general one."""
    from avr_amd.model import _bias_columns, _per_pose, _per_ray, _ray_pose_bias

    w = WORKLOADS[workload]
    cfg = dict(MESHRIR_MODEL, signal_output_dim=w.T)
    model = AVRModel(cfg, mlp_dtype=torch.bfloat16, enc_dtype=enc_dtype).to(DEV)
    with torch.no_grad():
        for enc in (model._dir_encoding, model._tx_encoding):
            enc.params.uniform_(-1, 1)
    B = 2
    r = AVRRender(model, **w.render)
    g = torch.Generator(device=DEV).manual_seed(4)
    pts, view, tx, _, geom = r.sample(torch.rand(B, 3, device=DEV, generator=g) * 4 - 2,
                                      torch.rand(B, 3, device=DEV, generator=g) * 4 - 2)
    L = (B, geom["n_rays"], w.n_samples)
    wd, wt = _bias_columns(model._model_signal.layers[0].weight)
    with torch.no_grad():
        got = _ray_pose_bias(model._dir_encoding, model._tx_encoding, view, tx, wd, wt, L)
        dir_e = model._dir_encoding((_per_ray(view.reshape(-1, 3), L) + 1) / 2)
        tx_e = model._tx_encoding((_per_pose(tx.reshape(-1, 3), L) + 1) / 2)
        ref = dir_e.to(torch.bfloat16).float() @ wd
        ref = (ref.view(B, L[1], -1) + (tx_e.to(torch.bfloat16).float() @ wt).view(B, 1, -1)).reshape(B * L[1], -1)
    assert got is not None and got.shape == ref.shape
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))
    with torch.no_grad():
        again = _ray_pose_bias(model._dir_encoding, model._tx_encoding, view, tx, wd, wt, L)
    assert torch.equal(got, again)


def test_unit_map_is_bit_identical():
    from avr_amd.model import _unit

    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.rand(1 << 20, 3, device=DEV, generator=g) * 2 - 1
    x[:4, 0] = torch.tensor([-1.0, 1.0, 0.0, -1 + 2 ** -24], device=DEV)
    assert torch.equal(_unit(x), (x + 1) / 2)


def test_head_takes_over_last_relu_backward(monkeypatch):
    """Training with the fused head: the head's backward applies the last
    hidden layer's ReLU mask (avr_head_bwd2 relu_mask) and the layer skips
    its threshold_backward.  The same selection on the same rounded values:
    every parameter gradient bitwise equal to the unlinked path
    (AVRRender(head_relu_link=False)), and the link was taken."""
    from avr_amd import model as M

    w = WORKLOADS["c1_meshrir_plumbing"].replace(name="raf_small", **{k: v for k, v in WORKLOADS[
        "c3_raf_furnished_b4"].render.items() if k not in ("n_azi", "n_ele", "n_samples")})
    w = w.replace(T=RAF_MODEL["signal_output_dim"], batch=2)
    torch.manual_seed(0)
    net = AVRModel_complex(RAF_MODEL, mlp_dtype=torch.bfloat16).to(DEV)
    r = AVRRender(net, **w.render).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(1)
    ro = torch.rand(w.batch, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(w.batch, 3, device=DEV, generator=g) * 2 - 1
    dtx = torch.nn.functional.normalize(torch.randn(w.batch, 3, device=DEV, generator=g), dim=-1)
    links = []
    orig = M.MLP.hidden
    monkeypatch.setattr(M.MLP, "hidden", lambda self, x, link=None: (links.append(link), orig(self, x, link))[1])
    grads = []
    for on in (True, False):
        r.head_relu_link = on
        r.zero_grad(set_to_none=True)
        torch.manual_seed(5)
        out = r(ro, tx, dtx)
        (out * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
        grads.append({n: p.grad.clone() for n, p in r.named_parameters() if p.grad is not None})
    torch.cuda.synchronize()
    signal_links = [l for l in links if l is not None]
    assert [l[0] for l in signal_links] == [True, False]
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 0
    bad = []
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        if "encoding" in n:
            # hash-grid tables: the small grids' backward adds with atomics
            # (fp32 order varies run to run), so equal up to that order
            rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
            if rel > 1e-5:
                bad.append((n, rel))
        elif not torch.equal(a, b):
            bad.append((n, float((a - b).abs().max())))
    assert not bad, bad


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("N,K", [(83200, 128), (1, 8), (1000, 512), (777, 64)])
def test_linear_out1_matches_torch(dtype, N, K, monkeypatch):
    """The one-output layer (avr_linear_out1_*) against the torch ops it
    replaces: forward within one 16-bit rounding of the fp64 sum (small
    integers: exact), data gradient bitwise equal to gy * w, weight gradient
    against fp64 (small integers: exact), deterministic."""
    from avr_amd import model as M

    gen = torch.Generator(device=DEV).manual_seed(N + K)
    x = torch.randint(-3, 4, (N, K), device=DEV, generator=gen).to(dtype).requires_grad_(True)
    wm = torch.randint(-2, 3, (1, K), device=DEV, generator=gen).float().requires_grad_(True)
    gy = torch.randint(-2, 3, (N, 1), device=DEV, generator=gen).to(dtype)
    assert M._out1_ok(x, wm, dtype)
    y = M._LinearOut1.apply(x, wm, dtype, False)
    y.backward(gy)
    ref_y = (x.detach().double() @ wm.detach().double().t()).to(dtype)
    assert torch.equal(y, ref_y)
    assert torch.equal(x.grad, gy * wm.detach().to(dtype))
    ref_gw = (gy.double().t() @ x.detach().double()).float()
    assert torch.equal(wm.grad, ref_gw)
    # random operands: bitwise repeatable; within rounding of fp64
    xr = torch.randn(N, K, device=DEV, generator=gen).to(dtype).requires_grad_(True)
    gr = torch.randn(N, 1, device=DEV, generator=gen).to(dtype)
    outs = []
    for _ in range(2):
        xr.grad = None
        wm.grad = None
        yr = M._LinearOut1.apply(xr, wm, dtype, False)
        yr.backward(gr)
        outs.append((yr.clone(), xr.grad.clone(), wm.grad.clone()))
    assert all(torch.equal(a, b) for a, b in zip(*outs))
    gw64 = gr.double().t() @ xr.detach().double()
    assert float((outs[0][2].double() - gw64).norm() / gw64.norm()) < 1e-5
