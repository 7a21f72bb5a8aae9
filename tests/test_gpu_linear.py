"""GPU: avr_linear_relu_fwd (csrc/linear_fwd.hip), the signal network's
width-512 hidden layers y = relu(x W^T) on the matrix cores, against a plain
PyTorch fp32 statement of the same layer rounded once to the 16-bit type
(model.py:176-180; tcnn's layers accumulate in fp32 and round their output).
Both sides round fp32 sums of exact 16-bit products, in different orders, so
elements may differ by one 16-bit ulp where the fp32 sums straddle a
rounding boundary."""
import ctypes

import pytest
import torch

from avr_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CODE = {torch.float16: _lib.DTYPE_F16, torch.bfloat16: _lib.DTYPE_BF16}


def _run(x, w, relu=True):
    M, K = x.shape
    N = w.size(0)
    y = torch.empty(M, N, dtype=x.dtype, device=DEV)
    wf = torch.empty_like(w)
    st = torch.cuda.current_stream(DEV).cuda_stream
    _lib.call("avr_linear_pack_w", N, K, w.data_ptr(), CODE[x.dtype], wf.data_ptr(), st)
    _lib.call("avr_linear_relu_fwd", M, N, K, x.data_ptr(), wf.data_ptr(), CODE[x.dtype],
              int(relu), y.data_ptr(), st)
    return y


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("M,N,relu", [(64, 256, True), (1000, 512, True), (4096 + 37, 512, False),
                                      (300, 96, True), (262144, 512, True)])
def test_linear_relu_matches_fp32_statement(dtype, M, N, relu):
    g = torch.Generator(device=DEV).manual_seed(M + N)
    x = torch.relu(torch.randn(M, 512, device=DEV, generator=g)).to(dtype)
    w = (torch.randn(N, 512, device=DEV, generator=g) / 512 ** 0.5).to(dtype)
    y = _run(x, w, relu)
    torch.cuda.synchronize()
    ref32 = x.float() @ w.float().t()
    if relu:
        ref32 = torch.relu(ref32)
    ref = ref32.to(dtype).float()
    yf = y.float()
    # one ulp of the rounded value, plus the fp32 summation-order error of
    # sums near zero (where the ReLU or the rounding can fall either way)
    ulp = torch.finfo(dtype).eps * ref.abs()
    tol = ulp * 1.01 + 1e-5 * (x.float().abs() @ w.float().abs().t())
    assert bool(((yf - ref).abs() <= tol).all()), float(((yf - ref).abs() - tol).max())
    assert float((yf != ref).float().mean()) < 0.02
    assert bool(torch.isfinite(yf).all())


def test_linear_relu_rejects_unsupported_shapes():
    x = torch.zeros(64, 256, dtype=torch.float16, device=DEV)
    w = torch.zeros(256, 256, dtype=torch.float16, device=DEV)
    y = torch.empty(64, 256, dtype=torch.float16, device=DEV)
    lib = _lib.load()
    p = ctypes.c_void_p
    assert lib.avr_linear_relu_fwd(64, 256, 256, p(x.data_ptr()), p(w.data_ptr()), _lib.DTYPE_F16, 1,
                                   p(y.data_ptr()), None) != 0  # K != 512
    assert lib.avr_linear_relu_fwd(64, 40, 512, p(x.data_ptr()), p(w.data_ptr()), _lib.DTYPE_F16, 1,
                                   p(y.data_ptr()), None) != 0  # N not a multiple of 32
    assert lib.avr_linear_pack_w(40, 512, p(w.data_ptr()), _lib.DTYPE_F16, p(y.data_ptr()), None) != 0
