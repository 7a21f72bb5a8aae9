"""GPU: avr_linear512_relu_fwd (csrc/linear512.hip), one width-512 ReLU
layer of the signal network (model.py:176-180), against a plain PyTorch fp32
statement of the same layer rounded once to the 16-bit type.

* Small-integer operands: every fp32 sum is exact whatever its order, so the
  kernel must equal the statement bit for bit, at row counts that leave
  partial row tiles, empty column-half pairings and several tiles per
  workgroup.
* Random operands: fp32 sums in another order; elements within a 16-bit
  ulp, a small share differing.
* Repeated launches are bitwise equal; the model path (AVR_LINEAR512=1)
  agrees with the hipBLASLt layers."""
import ctypes

import pytest
import torch

from avr_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CODE = {torch.float16: _lib.DTYPE_F16, torch.bfloat16: _lib.DTYPE_BF16}


def _run(x, w):
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    wf = torch.empty(512, 512, dtype=x.dtype, device=DEV)
    _lib.call("avr_linear512_pack_w", ctypes.c_void_p(w.data_ptr()), CODE[x.dtype], ctypes.c_void_p(wf.data_ptr()),
              st)
    y = torch.full_like(x, float("nan"))
    _lib.call("avr_linear512_relu_fwd", x.size(0), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(wf.data_ptr()),
              CODE[x.dtype], ctypes.c_void_p(y.data_ptr()), st)
    return y


def _ref(x, w):
    return torch.relu(x.float() @ w.float().t()).to(x.dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("M", [1, 255, 256, 257, 2048 + 7, 256 * 9, 100000, 262144])
def test_linear512_exact_on_integer_operands(dtype, M):
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randint(0, 3, (M, 512), device=DEV, generator=g).to(dtype)
    w = torch.randint(-1, 2, (512, 512), device=DEV, generator=g).to(dtype)
    y = _run(x, w)
    torch.cuda.synchronize()
    ref = _ref(x, w)
    assert torch.equal(y, ref), int((y != ref).sum())


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_linear512_random_operands_within_an_ulp(dtype):
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.relu(torch.randn(262144, 512, device=DEV, generator=g)).to(dtype)
    w = (torch.randn(512, 512, device=DEV, generator=g) / 512 ** 0.5).to(dtype)
    y = _run(x, w).float()
    ref = _ref(x, w).float()
    ulp = 2.0 ** -10 if dtype == torch.float16 else 2.0 ** -7
    err = (y - ref).abs() / torch.maximum(ref.abs(), ref.pow(2).mean().sqrt())
    assert torch.isfinite(y).all()
    assert float(err.max()) <= 2 * ulp, float(err.max())
    assert float((y != ref).float().mean()) < 0.02


def test_linear512_repeat_bitwise():
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.relu(torch.randn(300001, 512, device=DEV, generator=g)).half()
    w = (torch.randn(512, 512, device=DEV, generator=g) / 512 ** 0.5).half()
    a, b = _run(x, w), _run(x, w)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_mlp_hidden_on_linear512_matches_hipblaslt(dtype, monkeypatch):
    """MLP.hidden_from through the hand-written layers (AVR_LINEAR512=1) and
    through hipBLASLt: the same 16-bit rounding, fp32 sums in another order."""
    from avr_amd import model

    torch.manual_seed(1)
    mlp = model.MLP(512, 254, {"n_neurons": 512, "n_hidden_layers": 4}, dtype=dtype).to(DEV)
    x = torch.relu(torch.randn(40000, 512, device=DEV)).to(dtype)
    calls = []
    fn = model._linear512
    monkeypatch.setattr(model, "_linear512", lambda *a: calls.append(1) or fn(*a))
    outs = []
    for on in (True, False):
        monkeypatch.setattr(model, "_LINEAR512", on)
        with torch.no_grad():
            outs.append(mlp.hidden_from(x, 1).float())
    torch.cuda.synchronize()
    assert len(calls) == 3
    a, b = outs
    rel = float((a - b).norm() / b.norm())
    assert float(b.norm()) > 0 and rel < 1e-2, rel
