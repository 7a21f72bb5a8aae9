"""GPU: grouped feature concatenation (`csrc/concat.hip`) against the
expand + cat it replaces (forward: exact; backward: group sums in fp32 up
to summation order, deterministic), and inside the networks' training path
(KernelOptions(grouped_concat=False) vs True)."""
import pytest
import torch

from avr_amd.options import KernelOptions
from avr_amd.options import apply as apply_options

from avr_amd.concat import grouped_concat

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _reference(parts, N, out_dtype):
    cols = [t.repeat_interleave(d, 0).to(out_dtype) for t, d in parts]
    return torch.cat(cols, -1)


@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,R,S", [(2, 32, 64), (4, 650, 32), (1, 7, 3)])
def test_forward_and_backward_match_expand_cat(out_dtype, B, R, S):
    g = torch.Generator(device=DEV).manual_seed(0)
    N = B * R * S
    mk = lambda rows, w, dt: torch.randn(rows, w, device=DEV, generator=g).to(dt).requires_grad_(True)  # noqa: E731
    parts = [(mk(N, 256, torch.bfloat16), 1), (mk(B * R, 40, torch.float32), S),
             (mk(B, 40, torch.float16), R * S), (mk(N, 40, torch.float32), 1), (mk(B, 40, torch.float32), R * S)]
    out = grouped_concat(parts, N, out_dtype, splits=[1, 1, R, 1, R])
    ref = _reference([(t.detach(), d) for t, d in parts], N, out_dtype)
    assert torch.equal(out, ref)
    go = torch.randn(N, out.size(1), device=DEV, generator=g).to(out_dtype)
    grads = torch.autograd.grad(out, [t for t, _ in parts], go)
    again = torch.autograd.grad(grouped_concat(parts, N, out_dtype, splits=[1, 1, R, 1, R]),
                                [t for t, _ in parts], go)
    col = 0
    for (t, d), gr, g2 in zip(parts, grads, again):
        w = t.size(1)
        exp = go[:, col:col + w].float().view(-1, d, w).sum(1)
        col += w
        assert gr.dtype == t.dtype and gr.shape == t.shape
        assert torch.equal(gr, g2)  # deterministic
        tol = 1e-5 if t.dtype == torch.float32 else 1e-2
        torch.testing.assert_close(gr.float(), exp.to(t.dtype).float(), rtol=tol, atol=tol * max(1.0, d ** 0.5))


@pytest.mark.parametrize("cls", ["AVRModel", "AVRModel_complex"])
def test_network_training_path_matches_expand_cat(cls, monkeypatch):
    from avr_amd.model import AVRModel, AVRModel_complex
    from avr_amd.workloads import MESHRIR_MODEL, RAF_MODEL, WORKLOADS

    w = WORKLOADS["c1_meshrir_plumbing"]
    B, R, S = 2, w.n_rays, w.n_samples
    torch.manual_seed(0)
    if cls == "AVRModel":
        # fp32 encodings: the expand + cat path rounds the per-sample gradient
        # of fp16 encodings to fp16 before the group sum (small gradients
        # underflow there); grouped_concat sums the bf16 gradient in fp32
        m = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254), mlp_dtype=torch.bfloat16,
                     enc_dtype=torch.float32).to(DEV)
        extra = ()
    else:
        m = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=254), mlp_dtype=torch.bfloat16).to(DEV)
        extra = (torch.rand(B, 1, 3, device=DEV).expand(B, R * S, 3).contiguous() * 2 - 1,)
    with torch.no_grad():
        for p in m.parameters():
            if p.dim() == 1:
                p.uniform_(-1e-2, 1e-2)
    pts = torch.rand(B, R * S, 3, device=DEV) * 2 - 1
    view = torch.rand(B, R, 1, 3, device=DEV).expand(B, R, S, 3).reshape(B, R * S, 3) * 2 - 1
    tx = torch.rand(B, 1, 3, device=DEV).expand(B, R * S, 3).contiguous() * 2 - 1
    res = []
    for flag in (False, True):
        apply_options(m, KernelOptions(grouped_concat=flag))
        m.zero_grad()
        attn, sig = m(pts, view, tx, *extra, ray_layout=(B, R, S))
        (attn.float().sum() + sig.float().square().mean()).backward()
        res.append((attn.detach(), sig.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for n, g0 in res[0][2].items():
        g1 = res[1][2][n]
        err = float((g1 - g0).norm() / g0.norm().clamp_min(1e-30))
        assert err < 2e-3, (n, err)
