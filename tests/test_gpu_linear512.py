"""GPU: the hand-written MFMA layers of the MLP training path against plain
PyTorch fp32 statements of the same layers rounded once to the 16-bit type.

* avr_linear512_mask_fwd (csrc/linear512.hip): a width-512 layer's data
  gradient with the input ReLU's backward fused (model.py:176-180 trained
  through avr_runner.py:190), bit-exact on small-integer operands for every
  mask class, repeat-bitwise, and the MLP chain against the unfused one.
* avr_narrow_mm (csrc/mlp.hip): the RAF sigma encoder's narrow layers."""
import ctypes

import pytest
import torch

from avr_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CODE = {torch.float16: _lib.DTYPE_F16, torch.bfloat16: _lib.DTYPE_BF16}


# ---- the masked data gradient (avr_linear512_mask_fwd, W^T packing) ----

def _run_mask(g, w, mask):
    """0 where mask <= 0, else g W: W^T packed by avr_linear512_pack_w2."""
    st = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    wf = torch.empty(512, 512, dtype=g.dtype, device=DEV)
    _lib.call("avr_linear512_pack_w2", ctypes.c_void_p(w.data_ptr()), CODE[g.dtype], 1,
              ctypes.c_void_p(wf.data_ptr()), st)
    y = torch.full_like(g, float("nan"))
    _lib.call("avr_linear512_mask_fwd", g.size(0), ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(wf.data_ptr()),
              CODE[g.dtype], ctypes.c_void_p(mask.data_ptr()), ctypes.c_void_p(y.data_ptr()), st)
    return y


def _mask_values(M, dtype, gen):
    """Activations with every class threshold_backward distinguishes:
    positive, +0, -0, negative, +inf, -inf, NaN, the smallest subnormal."""
    m = torch.randn(M, 512, device=DEV, generator=gen).to(dtype)
    specials = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), -1.0], dtype=dtype, device=DEV)
    tiny = torch.tensor([1], dtype=torch.int16, device=DEV).view(dtype)  # smallest positive subnormal
    idx = torch.randint(0, 8, (M, 512), device=DEV, generator=gen)
    for i in range(6):
        m = torch.where(idx == i, specials[i], m)
    return torch.where(idx == 6, tiny, m).contiguous()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("M", [1, 257, 2048 + 7, 83200])
def test_masked_dgrad_exact_on_integer_operands(dtype, M):
    """Small-integer g and W: g W exact in fp32, so the kernel equals
    threshold_backward(g @ W, mask, 0) bit for bit, for every mask class."""
    gen = torch.Generator(device=DEV).manual_seed(M + 11)
    g = torch.randint(-2, 3, (M, 512), device=DEV, generator=gen).to(dtype)
    w = torch.randint(-1, 2, (512, 512), device=DEV, generator=gen).to(dtype)
    mask = _mask_values(M, dtype, gen)
    y = _run_mask(g, w, mask)
    torch.cuda.synchronize()
    ref = torch.ops.aten.threshold_backward((g.float() @ w.float()).to(dtype), mask, 0)
    assert torch.equal(y, ref), int((y != ref).sum())


def _integer_mlp(mlp, gen, density=16):
    """Weights in {-1, 0, 1}, one in `density` nonzero (no fp16 overflow in
    four layers): every fp32 sum of the
    chain is an exact integer, so any two summation orders agree bit for bit
    (values above the 16-bit types' integer range round the same way in both)."""
    with torch.no_grad():
        for p in mlp.parameters():
            v = torch.randint(-1, 2, p.shape, device=DEV, generator=gen).float()
            keep = torch.randint(0, density, p.shape, device=DEV, generator=gen) == 0
            p.copy_(v * keep)


def test_masked_dgrad_repeat_bitwise():
    gen = torch.Generator(device=DEV).manual_seed(21)
    g = torch.randn(83200, 512, device=DEV, generator=gen).half()
    w = (torch.randn(512, 512, device=DEV, generator=gen) / 512 ** 0.5).half()
    mask = _mask_values(83200, torch.float16, gen)
    a, b = _run_mask(g, w, mask), _run_mask(g, w, mask)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_mlp_training_chain_fused_dgrad(dtype):
    """MLP.hidden's backward with each ReLU's backward fused into the next
    layer's data gradient (KernelOptions.fused_dgrad, the default) against the
    unfused chain (hipBLASLt g @ W + threshold_backward) on small-integer
    operands: the same masks and exact fp32 sums, so every gradient is
    bitwise equal; the fused kernel is the one that ran."""
    from avr_amd import model
    from avr_amd.options import KernelOptions
    from avr_amd.options import apply as apply_options

    gen = torch.Generator(device=DEV).manual_seed(2)
    mlp = model.MLP(416, 64, {"n_neurons": 512, "n_hidden_layers": 4}, dtype=dtype).to(DEV)
    _integer_mlp(mlp, gen)
    x = torch.randint(-2, 3, (20000, 416), device=DEV, generator=gen).to(dtype).requires_grad_(True)
    calls = []
    fn = model._dgrad512_masked
    r = torch.randint(-2, 3, (20000, 64), device=DEV, generator=gen).float()
    grads = []
    orig = model._dgrad512_masked
    try:
        model._dgrad512_masked = lambda *a: calls.append(1) or fn(*a)
        for on in (True, False):
            apply_options(mlp, KernelOptions(fused_dgrad=on))
            mlp.zero_grad(set_to_none=True)
            x.grad = None
            out = mlp(x)
            (out.float() * r).sum().backward()
            grads.append([out.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in mlp.parameters()])
    finally:
        model._dgrad512_masked = orig
    torch.cuda.synchronize()
    assert len(calls) == 3  # layers 1..3 (512 x 512), not the 416-wide first
    for i, (a, b) in enumerate(zip(*grads)):
        assert float(b.float().norm()) > 0 and torch.equal(a, b), i


# ---- narrow layers (avr_narrow_mm) ----

@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
@pytest.mark.parametrize("N,R,C", [(83200, 128, 128), (83200, 80, 128), (83200, 128, 256), (83200, 256, 128),
                                   (83200, 128, 80), (1, 128, 128), (129, 256, 100), (777, 80, 68)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_narrow_mm_exact_on_integer_operands(dtype, N, R, C, act):
    """Small-integer operands (exact fp32 sums): equal to the fp32 statement
    rounded once, with no activation, ReLU, or threshold_backward's mask
    (every class: +-0, +-inf, NaN, subnormal)."""
    from avr_amd import model as M

    gen = torch.Generator(device=DEV).manual_seed(N + R + C + act)
    x = torch.randint(-2, 3, (N, R), device=DEV, generator=gen).to(dtype)
    bt = torch.randint(-1, 2, (C, R), device=DEV, generator=gen).to(dtype)
    mask = _mask_values(N, dtype, gen)[:, :C].contiguous() if C <= 512 else None
    y = M._narrow(x, bt, act, mask if act == 2 else None)
    torch.cuda.synchronize()
    ref = (x.float() @ bt.float().t()).to(dtype)
    if act == 1:
        ref = torch.relu(ref)
    elif act == 2:
        ref = torch.ops.aten.threshold_backward(ref, mask, 0)
    assert torch.equal(y, ref), int((y != ref).sum())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "fp16"])
def test_narrow_chain_training_matches_hipblaslt(dtype, monkeypatch):
    """The RAF sigma encoder's chain (80 -> 128 -> 128 -> 128 -> 256, ReLU on
    every layer) trained through avr_narrow_mm (forward + data gradients with
    the fused masks) against hipBLASLt + threshold_backward (narrow="off"):
    the same roundings, fp32 sums in another order."""
    from avr_amd import model as M

    torch.manual_seed(4)
    mlp = M.MLP(80, 256, {"n_neurons": 128, "n_hidden_layers": 3}, dtype=dtype).to(DEV)
    x = torch.randn(20000, 80, device=DEV).to(dtype).requires_grad_(True)
    r = torch.randn(20000, 256, device=DEV)
    calls = []
    fn = M._narrow
    monkeypatch.setattr(M, "_narrow", lambda *a: calls.append(a[2]) or fn(*a))
    res = []
    from avr_amd.options import KernelOptions
    from avr_amd.options import apply as apply_options

    for on in (True, False):
        apply_options(mlp, KernelOptions(narrow="all" if on else "off"))
        mlp.zero_grad(set_to_none=True)
        x.grad = None
        out = mlp(x, out_relu=True)
        (out.float() * r).sum().backward()
        res.append([out.float().detach(), x.grad.float()] + [p.grad.clone() for p in mlp.parameters()])
    torch.cuda.synchronize()
    assert sorted(calls) == [0] + [1] * 4 + [2] * 3  # 4 forwards, 3 masked data gradients, 1 plain
    for a, b in zip(*res):
        rel = float((a - b).norm() / b.norm())
        assert float(b.norm()) > 0 and rel < 2e-2, rel
