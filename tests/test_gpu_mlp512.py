"""GPU: avr_mlp512x2_fwd (csrc/mlp512.hip), two width-512 ReLU layers of the
signal network in one launch (model.py:176-180), against a plain PyTorch fp32
statement of the same two layers, each rounded once to the 16-bit type as
the unfused layers (and tcnn) round their outputs.

* Small-integer operands: every fp32 sum is exact whatever its order, so the
  kernel must equal the statement bit for bit (both layers, including the
  rounding of layer 2's large sums).
* Random operands: the fp32 sums are order-dependent; elements may differ by
  one 16-bit ulp where a sum straddles a rounding boundary, which then moves
  layer 2's sums by ~|w| ulp: within a few ulp of the output's RMS.
* The model path: AVRModel inference through the fused pair against the
  per-layer GEMMs (AVR_MLP512X2=0)."""
import ctypes

import pytest
import torch

from avr_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CODE = {torch.float16: _lib.DTYPE_F16, torch.bfloat16: _lib.DTYPE_BF16}


def _run(x, w1, w2):
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    wf = torch.empty(2, 512, 512, dtype=x.dtype, device=DEV)
    _lib.call("avr_mlp512x2_pack_w", ctypes.c_void_p(w1.data_ptr()), ctypes.c_void_p(w2.data_ptr()), CODE[x.dtype],
              ctypes.c_void_p(wf.data_ptr()), st)
    y = torch.full_like(x, float("nan"))
    _lib.call("avr_mlp512x2_fwd", x.size(0), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wf.data_ptr()),
              CODE[x.dtype], ctypes.c_void_p(y.data_ptr()), st)
    return y


def _ref(x, w1, w2):
    h = torch.relu(x.float() @ w1.float().t()).to(x.dtype)
    return torch.relu(h.float() @ w2.float().t()).to(x.dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("M", [1, 37, 128, 1000, 128 * 300 + 5, 262144])
def test_mlp512x2_exact_on_integer_operands(dtype, M):
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randint(0, 3, (M, 512), device=DEV, generator=g).to(dtype)
    w1 = torch.randint(-1, 2, (512, 512), device=DEV, generator=g).to(dtype)
    w2 = torch.randint(-1, 2, (512, 512), device=DEV, generator=g).to(dtype)
    y = _run(x, w1, w2)
    torch.cuda.synchronize()
    ref = _ref(x, w1, w2)
    assert torch.equal(y, ref), int((y != ref).sum())


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("M", [300, 262144])
def test_mlp512x2_random_operands_within_an_ulp(dtype, M):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x = torch.relu(torch.randn(M, 512, device=DEV, generator=g)).to(dtype)
    w1 = (torch.randn(512, 512, device=DEV, generator=g) / 512 ** 0.5).to(dtype)
    w2 = (torch.randn(512, 512, device=DEV, generator=g) / 512 ** 0.5).to(dtype)
    y = _run(x, w1, w2).float()
    ref = _ref(x, w1, w2).float()
    ulp = 2.0 ** -10 if dtype == torch.float16 else 2.0 ** -7
    # an element of layer 1 that rounds the other way moves every layer-2
    # sum by ~|w| ulp(h): bounded relative to the output's scale, not to a
    # small element's own magnitude
    scale = ref.pow(2).mean().sqrt()
    err = (y - ref).abs() / torch.maximum(ref.abs(), scale)
    assert torch.isfinite(y).all()
    assert float(err.max()) <= 4 * ulp, float(err.max())
    assert float((y != ref).float().mean()) < 0.02


def test_mlp512x2_repeat_bitwise():
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.relu(torch.randn(70000, 512, device=DEV, generator=g)).half()
    w1 = (torch.randn(512, 512, device=DEV, generator=g) / 512 ** 0.5).half()
    w2 = (torch.randn(512, 512, device=DEV, generator=g) / 512 ** 0.5).half()
    a, b = _run(x, w1, w2), _run(x, w1, w2)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_mlp_hidden_from_fused_pairs_match_per_layer(dtype, monkeypatch):
    """MLP.hidden_from (the signal network's hidden layers after the fused
    first layer, model.py) through the fused pairs and per layer: same
    16-bit rounding, fp32 sums in a different order."""
    from avr_amd import model

    torch.manual_seed(1)
    mlp = model.MLP(512, 254, {"n_neurons": 512, "n_hidden_layers": 5}, dtype=dtype).to(DEV)
    x = torch.relu(torch.randn(5000, 512, device=DEV)).to(dtype)
    calls = []
    fused_fn = model._mlp512x2
    monkeypatch.setattr(model, "_mlp512x2", lambda *a: calls.append(1) or fused_fn(*a))
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(model, "_MLP512X2", fused)
        with torch.no_grad():
            outs.append(mlp.hidden_from(x, 1).float())
    torch.cuda.synchronize()
    assert len(calls) == 2  # layers 1-2 and 3-4 fused
    a, b = outs
    rel = float((a - b).norm() / b.norm())
    assert float(b.norm()) > 0 and rel < 1e-2, rel


def test_avrmodel_inference_fused_pair_matches_per_layer(monkeypatch):
    """The renderer's network output (c1 plumbing workload) through the fused
    pair and through the per-layer GEMMs agree to the 16-bit rounding."""
    from avr_amd import AVRRender, model
    from avr_amd.model import AVRModel
    from avr_amd.workloads import MESHRIR_MODEL, WORKLOADS

    w = WORKLOADS["c1_meshrir_plumbing"].replace(T=1022)
    torch.manual_seed(0)
    net = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=w.T), mlp_dtype=torch.bfloat16).to(DEV)
    r = AVRRender(net, **w.render).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(2)
    ro = torch.rand(1, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(1, 3, device=DEV, generator=g) * 2 - 1
    calls = []
    fused_fn = model._mlp512x2
    monkeypatch.setattr(model, "_mlp512x2", lambda *a: calls.append(1) or fused_fn(*a))
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(model, "_MLP512X2", fused)
        torch.manual_seed(3)
        with torch.no_grad():
            outs.append(r(ro, tx))
    torch.cuda.synchronize()
    a, b = outs
    assert calls, "the fused pair was not used"
    rel = float((a - b).norm() / b.norm())
    assert float(b.norm()) > 0 and torch.isfinite(a).all() and rel < 2e-2, rel
