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
    # short items: one and two 64-t tiles per work item (the shape class that
    # corrupted the round-4 bf16x3 DFT), oracle parity + repeats
    # (a lower fs keeps the receiver delay within the short IR's path-loss table)
    ("one_tile_k512", dict(MESHRIR, fs=4000), 6, 5, 32, 62, 512, 2),
    ("two_tiles_k512", dict(MESHRIR, fs=6000, xyz_min=0, xyz_max=10), 7, 4, 24, 126, 512, 3),
    # ray counts for every form of the delay sort: 1154 rays (config 4's
    # RAF-E sphere) sort 2048 keys, 2562 rays 4096 keys, 8 keys per thread /
    # 16 keys per thread in registers (650 and 1024 rays above: 4)
    ("raf_e_rays", RAF, 48, 24, 16, 510, 64, 1),
    ("many_rays", MESHRIR, 64, 40, 8, 254, 64, 1),
    # K % 8 != 0: the backward's scan form (csrc/head.hip head_bwd_h_kernel;
    # every other case takes the block-sum form); no exact head
    # for K % 16 != 0, so only the linear forms run it
    ("k12_scan_bwd", SIMU, 8, 4, 24, 4094, 12, 1),  # (T > 2048: feature blocks of 4)
]


def _skip_inexact(case, exact):
    if exact and case[6] % 16:
        pytest.skip("the exact head takes K % 16 == 0")


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


def _round16(x, dtype, exact=True):
    """The value the unfused layer outputs: x rounded to the 16-bit MLP dtype
    (the reference network's fp16 output), gradient passed straight through
    (as through the unfused layer's rounding)."""
    if not exact or dtype == torch.float32:
        return x
    return x + (x.to(dtype).float() - x).detach()


def _fused(case, dtype, ops=None, exact=True):
    """Fused render + backward; returns (out, grad_attn, grad_h, grad_W)."""
    cfg, ro, tx, attn, h, W, go = ops or _operands(case, dtype)
    r = AVRRender(None, exact_head=exact, **cfg)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    a1 = attn.clone().requires_grad_(True)
    h1 = h.clone().requires_grad_(True)
    W1 = W.clone().requires_grad_(True)
    out = r.render_from_hidden(a1, h1, W1, dtype, geom)
    (out * go).sum().backward()
    return out.detach(), a1.grad, h1.grad, W1.grad


HEAD_FORMS = [(torch.float32, False), (torch.bfloat16, True), (torch.float16, True),
              (torch.bfloat16, False), (torch.float16, False)]
HEAD_IDS = ["fp32", "bf16-exact", "fp16-exact", "bf16-linear", "fp16-linear"]


@pytest.mark.parametrize("dtype,exact", HEAD_FORMS, ids=HEAD_IDS)
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_matches_oracle(case, dtype, exact):
    """Fused head against the CPU oracle (the reference's algorithm) on the
    signal the reference renders: h @ W^T of the dtype-rounded operands,
    rounded to the 16-bit MLP dtype for a 16-bit network (the default exact
    head; the linear head, exact=False, against the unrounded product),
    forward and backward.  The backward of both forms differentiates the
    unrounded product, so for the exact form the gradients to attn differ
    from the rounded signal's by the 16-bit rounding (bar 3e-3 at bf16)."""
    _skip_inexact(case, exact)
    name = case[0]
    ops = _operands(case, dtype)
    cfg, ro, tx, attn, h, W, go = ops
    out_f, ga_f, gh_f, gW_f = _fused(case, dtype, ops, exact)

    hc = h.float().cpu()
    Wc = W.to(dtype).float().cpu().double()
    ac = attn.cpu().requires_grad_(True)
    sig = (hc.double() @ Wc.t()).float()
    if exact:
        sig = sig.to(dtype).float()
    sig = sig.requires_grad_(True)
    torch.manual_seed(5)  # the jitter draw the fused render consumed
    ref = orc.render_spectrum(orc.RenderConfig.from_kwargs(**cfg), orc.StubNetwork(ac, sig),
                              ro.cpu(), tx.cpu())
    (ref * go.cpu()).sum().backward()
    gs = sig.grad.double()
    gh_ref = gs @ Wc  # dL/dh = dL/dsignal @ W
    gW_ref = torch.einsum("brt,brk->tk", gs, hc.double())  # dL/dW = sum over rows

    assert _rel(out_f.cpu(), ref) < 1e-4, (name, _rel(out_f.cpu(), ref))
    tol_h = 1e-3 if dtype == torch.float32 else 6e-3  # grad_h is stored in the h dtype
    tol_a = 3e-3 if (exact and dtype == torch.bfloat16) else 1e-3
    assert _rel(ga_f.cpu(), ac.grad) < tol_a, (name, "attn", _rel(ga_f.cpu(), ac.grad))
    assert _rel(gh_f.float().cpu(), gh_ref) < tol_h, (name, "h", _rel(gh_f.float().cpu(), gh_ref))
    assert _rel(gW_f.cpu(), gW_ref) < 1e-3, (name, "W", _rel(gW_f.cpu(), gW_ref))


@pytest.mark.parametrize("dtype,exact", HEAD_FORMS, ids=HEAD_IDS)
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_bitwise_reproducible(case, dtype, exact):
    """Two renders (forward + backward) of the same operands are identical."""
    _skip_inexact(case, exact)
    ops = _operands(case, dtype)
    a = _fused(case, dtype, ops, exact)
    b = _fused(case, dtype, ops, exact)
    for x, y, what in zip(a, b, ("out", "grad_attn", "grad_h", "grad_W")):
        assert torch.equal(x, y), (case[0], what)


@pytest.mark.parametrize("dtype,exact", HEAD_FORMS, ids=HEAD_IDS)
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_matches_plain_render(case, dtype, exact):
    """The fused head against the plain (golden-pinned) render of the
    signal the unfused layer produces: the fp32 product, rounded to the
    16-bit dtype for the exact form."""
    _skip_inexact(case, exact)
    name, base, n_azi, n_ele, S, T, K, B = case
    cfg, ro, tx, attn, h, W, go = _operands(case, dtype)
    r = AVRRender(None, exact_head=exact, **cfg)
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
    sig = _round16(h2.float() @ W2.t(), dtype, exact)
    out_u = r.render_from_network_output(a2, sig, geom)

    assert _rel(out_f, out_u) < 2e-5, (name, _rel(out_f, out_u))
    (out_f * go).sum().backward()
    (out_u * go).sum().backward()
    tol_h = 2e-4 if dtype == torch.float32 else 6e-3  # grad_h is stored in the h dtype
    # exact form: the backward differentiates the unrounded product (see
    # test_fused_head_matches_oracle), the plain render the rounded signal
    tol_a = 2e-4 if not exact else (3e-3 if dtype == torch.bfloat16 else 1e-3)
    assert _rel(a1.grad, a2.grad) < tol_a, (name, "attn", _rel(a1.grad, a2.grad))
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
    the 16-bit layer's output: h @ W^T on the same 16-bit operands, fp32
    accumulation, every element rounded to the MLP dtype (the exact head)."""
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
        sig = (h.float() @ weight.to(dtype).float().t()).to(dtype).float()  # the 16-bit layer's output
        plain = r.render_from_network_output(attn, sig, geom)
        torch.manual_seed(3)
        end_to_end = r(ro, tx, dtx)  # the module's forward takes the fused path
    assert _rel(fused, plain) < 2e-5, _rel(fused, plain)
    assert torch.equal(end_to_end, fused)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_fused_head_config2_full_size(dtype):
    """Config 2 at full size (1024 rays x 256 samples x T=1022, K=512): the
    exact fused head against the plain render of the 16-bit layer output
    (h @ W^T rounded to the dtype), the linear head against the plain render
    of the unrounded product; repeat renders equal."""
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
        plain = r.render_from_network_output(attn, (h.float() @ W.to(dtype).float().t()).to(dtype).float(), geom)
        linear = AVRRender(None, exact_head=False, **w.render).render_from_hidden(attn, h, W, dtype, geom)
        exact_prod = r.render_from_network_output(attn, h.float() @ W.to(dtype).float().t(), geom)
    assert _rel(linear, exact_prod) < 2e-5, _rel(linear, exact_prod)
    assert torch.equal(fused, again)
    assert _rel(fused, plain) < 2e-5, _rel(fused, plain)


def test_fused_head_one_ray_shard():
    """A shard of ONE ray (ray_range of width 1: no sort pass runs, the
    delay-count scan alone orders the LDS) equals the plain render of
    h @ W^T for the same ray."""
    cfg = dict(MESHRIR, n_azi=6, n_ele=5, n_samples=64)
    T, K, B = 254, 64, 2
    R = 1
    g = torch.Generator(device=DEV).manual_seed(41)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    attn = torch.rand(B, R * 64, 1, device=DEV, generator=g) * 2
    h = torch.relu(torch.randn(B, R * 64, K, device=DEV, generator=g)).to(torch.bfloat16)
    W = torch.randn(T, K, device=DEV, generator=g) / K ** 0.5
    for r0 in (0, 7, 31):
        r = AVRRender(None, **cfg)
        r.ray_range = (r0, r0 + 1)
        torch.manual_seed(5)
        _, _, _, _, geom = r.sample(ro, tx)
        assert geom["n_rays"] == 1
        with torch.no_grad():
            fused = r.render_from_hidden(attn, h, W, torch.bfloat16, geom)
            again = r.render_from_hidden(attn, h, W, torch.bfloat16, geom)
            plain = r.render_from_network_output(
                attn, (h.float() @ W.to(torch.bfloat16).float().t()).to(torch.bfloat16).float(), geom)
        assert torch.equal(fused, again), r0
        if plain.abs().max() == 0:
            assert fused.abs().max() == 0, r0
        else:
            assert _rel(fused, plain) < 2e-5, (r0, _rel(fused, plain))


def test_fused_head_propagate_nonfinite():
    """propagate_nonfinite=True on the fused-head path: a NaN in the hidden
    row of a ray-sample whose window is empty (the head kernels never read
    it) leaves the default render clean but poisons the strict one, as the
    reference's signal = h W^T does through its masks (renderer.py:82,89)."""
    case = CASES[0]
    cfg, ro, tx, attn, h, W, go = _operands(case, torch.float16)
    r = AVRRender(None, **cfg)
    strict = AVRRender(None, propagate_nonfinite=True, **cfg)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    with torch.no_grad():
        clean = r.render_from_hidden(attn, h, W, torch.float16, geom)
        assert torch.isfinite(clean).all()
        assert torch.equal(strict.render_from_hidden(attn, h, W, torch.float16, geom), clean)
        # find a ray-sample the render never reads: NaN in its row changes nothing
        found = None
        for i in range(0, h.size(1), 7):
            hb = h.clone()
            hb[0, i, 0] = float("nan")
            if torch.equal(r.render_from_hidden(attn, hb, W, torch.float16, geom), clean):
                found = hb
                break
        assert found is not None, "no masked ray-sample in the test case"
        poisoned = strict.render_from_hidden(attn, found, W, torch.float16, geom)
    assert torch.isnan(poisoned).all()


def test_fused_head_config2_fp16_matches_oracle_rounded_signal():
    """Config 2 at full size with an fp16 network (tcnn's precision): the
    default (exact) fused head against the CPU oracle rendering
    signal = fp16(h @ W^T).float() -- what the reference renders from a
    16-bit network (renderer_cpu.py:73,80,90) -- at the north-star 1e-4.
    The linear head (exact_head=False) sums the unrounded products; its
    distance to the same oracle is reported, not bounded."""
    from avr_amd.workloads import WORKLOADS

    w = WORKLOADS["c2_meshrir_1024x256x512"]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, 512
    dtype = torch.float16
    g = torch.Generator(device=DEV).manual_seed(19)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=DEV, generator=g)).to(dtype)
    W = torch.randn(T, K, device=DEV, generator=g) / K ** 0.5
    r = AVRRender(None, **w.render)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    with torch.no_grad():
        exact = r.render_from_hidden(attn, h, W, dtype, geom).cpu()
        linear = AVRRender(None, exact_head=False, **w.render).render_from_hidden(attn, h, W, dtype, geom).cpu()
        sig = (h.float() @ W.to(dtype).float().t()).to(dtype).float().cpu()  # the 16-bit layer's output
    torch.manual_seed(5)
    ref = orc.render_spectrum(orc.RenderConfig.from_kwargs(**w.render), orc.StubNetwork(attn.cpu(), sig),
                              ro.cpu(), tx.cpu())
    e_exact, e_linear = _rel(exact, ref), _rel(linear, ref)
    emax = float((exact - ref).abs().max() / ref.abs().max())
    assert e_exact < 1e-4 and emax < 1e-4, (e_exact, emax, e_linear)


# K = 512 with more rays than one 256-ray slab of the exact head holds:
# config 4's RAF-E sphere (1154 rays: 5 slabs, n_split 8) and config 5's
# full 89 x 46 + 2 = 4096-ray sphere (16 slabs)
MANY_RAY_CASES = [
    ("raf_e_k512", RAF, 48, 24, 16, 510, 512, 2),
    ("sphere4096_k512", SIMU, 89, 46, 8, 254, 512, 1),
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("case", MANY_RAY_CASES, ids=[c[0] for c in MANY_RAY_CASES])
def test_exact_head_many_rays(case, dtype):
    """The exact head with K = 512 beyond 1024 rays: against the CPU oracle
    on the rounded signal (1e-4, L2 and max-norm) and the plain render of it
    (2e-5); repeat renders bitwise equal."""
    cfg, ro, tx, attn, h, W, _ = _operands(case, dtype)
    r = AVRRender(None, **cfg)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    with torch.no_grad():
        fused = r.render_from_hidden(attn, h, W, dtype, geom)
        again = r.render_from_hidden(attn, h, W, dtype, geom)
        sig = (h.float() @ W.to(dtype).float().t()).to(dtype).float()
        plain = r.render_from_network_output(attn, sig, geom)
    assert torch.equal(fused, again)
    assert _rel(fused, plain) < 2e-5, (case[0], _rel(fused, plain))
    torch.manual_seed(5)
    ref = orc.render_spectrum(orc.RenderConfig.from_kwargs(**cfg), orc.StubNetwork(attn.cpu(), sig.cpu()),
                              ro.cpu(), tx.cpu())
    assert _rel(fused.cpu(), ref) < 1e-4, (case[0], _rel(fused.cpu(), ref))
    assert float((fused.cpu() - ref).abs().max() / ref.abs().max()) < 1e-4
