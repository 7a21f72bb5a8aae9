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
