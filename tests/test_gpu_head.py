"""GPU: the fused signal head (csrc/head.hip).

The fused path never materialises the signal; by linearity it must equal the
reference render of signal = h @ W^T.  Checked two ways on the same operands:
* against the CPU oracle (oracle/avr_oracle.py, pinned bit-identical to
  renderer_cpu.py) on signal = h.float() @ W.T computed on the host, forward
  (1e-4, the north-star bar) and backward through oracle autograd (grads to
  attn, h = grad_signal @ W and W = grad_signal^T @ h);
* against the plain HIP render of the same product (tighter: 2e-5).
Renders and gradients are bitwise reproducible run to run."""
import pytest
import torch

from oracle import avr_oracle as orc

from avr_amd import AVRRender
from avr_amd.model import AVRModel_complex
from avr_amd.workloads import MESHRIR, RAF, RAF_MODEL, SIMU

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


CASES = [
    # name, render cfg, n_azi, n_ele, S, T, K, B
    ("meshrir_small", MESHRIR, 6, 5, 64, 254, 64, 2),
    ("raf_c3_like", RAF, 36, 18, 32, 1600, 512, 1),
    ("simu_long_T", SIMU, 8, 4, 48, 4094, 128, 1),
    ("meshrir_odd", dict(MESHRIR, xyz_min=0, xyz_max=10), 5, 3, 40, 510, 96, 3),
    # K = 512: the reference networks' width (model.py:176-180)
    ("meshrir_k512", MESHRIR, 16, 8, 64, 1022, 512, 2),
    ("simu_long_k512", SIMU, 8, 4, 48, 4094, 512, 1),
    ("ragged_k512", dict(MESHRIR, xyz_min=0, xyz_max=10), 5, 3, 40, 510, 512, 3),
    # ray counts for every form of the delay sort: 1154 rays (config 4's
    # RAF-E sphere) sort 2048 keys, 2562 rays 4096 keys, 8 keys per thread /
    # 16 keys per thread in registers (650 and 1024 rays above: 4)
    ("raf_e_rays", RAF, 48, 24, 16, 510, 64, 1),
    ("many_rays", MESHRIR, 64, 40, 8, 254, 64, 1),
]


def _operands(case, dtype):
    name, base, n_azi, n_ele, S, T, K, B = case
    cfg = dict(base, n_azi=n_azi, n_ele=n_ele, n_samples=S)
    R = n_azi * n_ele + 2
    g = torch.Generator(device=DEV).manual_seed(sum(map(ord, name)))
    ro = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    attn = (torch.rand(B, R * S, 1, device=DEV, generator=g) * 2)
    h = torch.relu(torch.randn(B, R * S, K, device=DEV, generator=g)).to(dtype)
    W = (torch.randn(T, K, device=DEV, generator=g) / K ** 0.5)
    go = torch.randn(B, T // 2 + 1, 2, device=DEV, generator=g)
    return cfg, ro, tx, attn, h, W, go


def _fused(case, dtype, ops=None):
    """Fused render + backward; returns (out, grad_attn, grad_h, grad_W)."""
    cfg, ro, tx, attn, h, W, go = ops or _operands(case, dtype)
    r = AVRRender(None, **cfg)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    a1 = attn.clone().requires_grad_(True)
    h1 = h.clone().requires_grad_(True)
    W1 = W.clone().requires_grad_(True)
    out = r.render_from_hidden(a1, h1, W1, dtype, geom)
    (out * go).sum().backward()
    return out.detach(), a1.grad, h1.grad, W1.grad


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_matches_oracle(case, dtype):
    """Fused head against the CPU oracle (the reference's algorithm) on
    signal = h @ W^T with the dtype-rounded operands, forward and backward."""
    name = case[0]
    ops = _operands(case, dtype)
    cfg, ro, tx, attn, h, W, go = ops
    out_f, ga_f, gh_f, gW_f = _fused(case, dtype, ops)

    hc = h.float().cpu()
    Wc = W.to(dtype).float().cpu().double()
    ac = attn.cpu().requires_grad_(True)
    sig = (hc.double() @ Wc.t()).float().requires_grad_(True)
    torch.manual_seed(5)  # the jitter draw the fused render consumed
    ref = orc.render_spectrum(orc.RenderConfig.from_kwargs(**cfg), orc.StubNetwork(ac, sig),
                              ro.cpu(), tx.cpu())
    (ref * go.cpu()).sum().backward()
    gs = sig.grad.double()
    gh_ref = gs @ Wc  # dL/dh = dL/dsignal @ W
    gW_ref = torch.einsum("brt,brk->tk", gs, hc.double())  # dL/dW = sum over rows

    assert _rel(out_f.cpu(), ref) < 1e-4, (name, _rel(out_f.cpu(), ref))
    tol_h = 1e-3 if dtype == torch.float32 else 6e-3  # grad_h is stored in the h dtype
    assert _rel(ga_f.cpu(), ac.grad) < 1e-3, (name, "attn", _rel(ga_f.cpu(), ac.grad))
    assert _rel(gh_f.float().cpu(), gh_ref) < tol_h, (name, "h", _rel(gh_f.float().cpu(), gh_ref))
    assert _rel(gW_f.cpu(), gW_ref) < 1e-3, (name, "W", _rel(gW_f.cpu(), gW_ref))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_bitwise_reproducible(case, dtype):
    """Two renders (forward + backward) of the same operands are identical."""
    ops = _operands(case, dtype)
    a = _fused(case, dtype, ops)
    b = _fused(case, dtype, ops)
    for x, y, what in zip(a, b, ("out", "grad_attn", "grad_h", "grad_W")):
        assert torch.equal(x, y), (case[0], what)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_matches_plain_render(case, dtype):
    name, base, n_azi, n_ele, S, T, K, B = case
    cfg, ro, tx, attn, h, W, go = _operands(case, dtype)
    r = AVRRender(None, **cfg)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)

    a1 = attn.clone().requires_grad_(True)
    h1 = h.clone().requires_grad_(True)
    W1 = W.clone().requires_grad_(True)
    out_f = r.render_from_hidden(a1, h1, W1, dtype, geom)

    a2 = attn.clone().requires_grad_(True)
    h2 = h.clone().requires_grad_(True)
    # the layer in fp32 on the same (dtype-rounded) operands; W's gradient
    # kept in fp32 as the fused path returns it to the fp32 master weight
    W2 = W.to(dtype).float().requires_grad_(True)
    sig = h2.float() @ W2.t()
    out_u = r.render_from_network_output(a2, sig, geom)

    assert _rel(out_f, out_u) < 2e-5, (name, _rel(out_f, out_u))
    (out_f * go).sum().backward()
    (out_u * go).sum().backward()
    tol_h = 2e-4 if dtype == torch.float32 else 6e-3  # grad_h is stored in the h dtype
    assert _rel(a1.grad, a2.grad) < 2e-4, (name, "attn", _rel(a1.grad, a2.grad))
    assert _rel(h1.grad, h2.grad) < tol_h, (name, "h", _rel(h1.grad, h2.grad))
    assert _rel(W1.grad, W2.grad) < 2e-4, (name, "W", _rel(W1.grad, W2.grad))
    # rows whose delay window is empty get exactly zero gradient
    assert torch.isfinite(h1.grad.float()).all()


def test_fused_head_model_matches_unfused():
    """AVRModel_complex (fp32 MLP) rendered with and without the fused head."""
    cfg = dict(RAF, n_azi=6, n_ele=5, n_samples=32)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800)).to(DEV)
    B = 2
    g = torch.Generator(device=DEV).manual_seed(11)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
    outs, grads = [], []
    for fused in (False, True):
        r = AVRRender(model, fused_head=fused, **cfg)
        model.zero_grad(set_to_none=True)
        torch.manual_seed(3)
        out = r(ro, tx, dtx)
        (out * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
        outs.append(out.detach())
        grads.append({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    assert _rel(outs[1], outs[0]) < 2e-5, _rel(outs[1], outs[0])
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        assert _rel(grads[1][n], grads[0][n]) < 5e-4, (n, _rel(grads[1][n], grads[0][n]))


def test_fused_head_falls_back_when_unsupported():
    """T above the fused kernels' limit: the network applies its last layer
    and the plain path renders (same result as fused_head=False)."""
    cfg = dict(SIMU, n_azi=4, n_ele=2, n_samples=16)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=4600)).to(DEV)
    B = 1
    ro = torch.zeros(B, 3, device=DEV)
    tx = torch.full((B, 3), 0.5, device=DEV)
    dtx = torch.tensor([[0.0, 0.0, 1.0]], device=DEV)
    torch.manual_seed(0)
    a = AVRRender(model, **cfg)(ro, tx, dtx)
    torch.manual_seed(0)
    b = AVRRender(model, fused_head=False, **cfg)(ro, tx, dtx)
    assert torch.equal(a, b)


@pytest.mark.parametrize("mlp_dtype", [torch.float16, torch.bfloat16])
def test_fused_head_model_reference_precision(mlp_dtype):
    """AVRModel_complex with 16-bit MLPs (fp16 is tcnn's precision,
    model.py:21-31) stays on the fused path and equals the plain render of
    the layer's exact product h @ W^T on the same 16-bit operands (fp32
    accumulation, as the fused head sums; rounding that product back to
    16 bits, as the unfused layer does, would only lose precision)."""
    cfg = dict(RAF, n_azi=6, n_ele=5, n_samples=32)
    torch.manual_seed(2)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800), mlp_dtype=mlp_dtype).to(DEV)
    B = 2
    g = torch.Generator(device=DEV).manual_seed(12)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
    r = AVRRender(model, **cfg)
    with torch.no_grad():
        torch.manual_seed(3)
        pts, view, txn, dtxn, geom = r.sample(ro, tx, dtx)
        # the ray layout the renderer passes (per-ray/per-pose first-layer
        # bias: its sums may round h one ulp apart from the plain trunk)
        layout = (B, geom["n_rays"], cfg["n_samples"])
        attn, h, weight, dtype = model.forward_fused(pts, view, txn, dtxn, ray_layout=layout)
        assert dtype == mlp_dtype and h.dtype == mlp_dtype and r._head_supported(geom, h, weight, dtype)
        fused = r.render_from_hidden(attn, h, weight, dtype, geom)
        sig = h.float() @ weight.to(dtype).float().t()
        plain = r.render_from_network_output(attn, sig, geom)
        torch.manual_seed(3)
        end_to_end = r(ro, tx, dtx)  # the module's forward takes the fused path
    assert _rel(fused, plain) < 2e-5, _rel(fused, plain)
    assert torch.equal(end_to_end, fused)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_fused_head_config2_full_size(dtype):
    """Config 2 at full size (1024 rays x 256 samples x T=1022, K=512): the
    fused head against the plain render of h @ W^T; repeat renders equal."""
    from avr_amd.workloads import WORKLOADS

    w = WORKLOADS["c2_meshrir_1024x256x512"]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, 512
    g = torch.Generator(device=DEV).manual_seed(9)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=DEV, generator=g)).to(dtype)
    W = torch.randn(T, K, device=DEV, generator=g) / K ** 0.5
    r = AVRRender(None, **w.render)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    with torch.no_grad():
        fused = r.render_from_hidden(attn, h, W, dtype, geom)
        again = r.render_from_hidden(attn, h, W, dtype, geom)
        plain = r.render_from_network_output(attn, h.float() @ W.to(dtype).float().t(), geom)
    assert torch.equal(fused, again)
    assert _rel(fused, plain) < 2e-5, _rel(fused, plain)
