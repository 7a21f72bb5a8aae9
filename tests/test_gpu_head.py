"""GPU: the fused signal head (csrc/head.hip) against
the plain render of signal = h @ W^T.

The fused path never materialises the signal; by linearity it must equal the
unfused render of the same network output, forward and backward (grads to
attn, h and W).  The reference for each case is the plain HIP path on the
fp32 product of the same operands (the plain path itself is pinned to the
reference's golden vectors in test_gpu_render.py)."""
import pytest
import torch

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
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_fused_head_matches_plain_render(case, dtype):
    name, base, n_azi, n_ele, S, T, K, B = case
    cfg = dict(base, n_azi=n_azi, n_ele=n_ele, n_samples=S)
    r = AVRRender(None, **cfg)
    R = n_azi * n_ele + 2
    g = torch.Generator(device=DEV).manual_seed(sum(map(ord, name)))
    ro = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    attn = (torch.rand(B, R * S, 1, device=DEV, generator=g) * 2)
    h = torch.relu(torch.randn(B, R * S, K, device=DEV, generator=g)).to(dtype)
    W = (torch.randn(T, K, device=DEV, generator=g) / K ** 0.5)

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
    go = torch.randn(out_f.shape, device=DEV, generator=g)
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
