"""The shipped TunableOp results for the width-512 hidden layers
(avr_amd/tunableop_gfx950.csv, avr_amd/model.py::_enable_tuned_gemms): file
format and the loader's guards on the CPU; on the GPU, the tuned solution's
output against the default hipBLASLt solution's, bit for bit."""
import csv
import os

import pytest
import torch

from avr_amd import model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_results_file_format():
    """Validators pin the libraries and gfx950; one entry per MLP dtype for
    the config-2 inference shape (M = 262,144 rows, 512 -> 512)."""
    rows = list(csv.reader(open(model._TUNED_FILE)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    for k in ("PT_VERSION", "HIP_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION"):
        assert k in val
    ops = {r[0]: r[1:] for r in rows if r[0] != "Validator"}
    for dt in ("Half", "BFloat16"):
        sig, sol, ms = ops[f"GemmAndBiasTunableOp_{dt}_TN"]
        assert sig == "tn_512_262144_512_ld_512_512_512" and sol.startswith("Gemm_") and float(ms) > 0


def test_loader_respects_opt_out(monkeypatch):
    """AVR_TUNABLEOP=0 returns before touching TunableOp or the device (on
    this CPU-only container any such call would raise)."""
    monkeypatch.setattr(model, "_TUNED", [False])
    monkeypatch.setenv("AVR_TUNABLEOP", "0")
    model._enable_tuned_gemms(torch.device("cpu"))
    assert model._TUNED[0]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_tuned_layer_bit_identical(dtype):
    """relu(x W^T) through _LinearReLU with the shipped solution equals the
    default hipBLASLt solution's output bit for bit (TunableOp off)."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.relu(torch.randn(262144, 512, device=dev, generator=g)).to(dtype)
    w = torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5
    bias = torch.zeros(512, dtype=dtype, device=dev)
    was = torch.cuda.tunable.is_enabled()
    torch.cuda.tunable.enable(False)
    ref = torch._addmm_activation(bias, x, w.to(dtype).t(), use_gelu=False)
    torch.cuda.tunable.enable(was)
    model._enable_tuned_gemms(dev)
    with torch.no_grad():
        y = model._LinearReLU.apply(x, w, dtype)
    if os.environ.get("AVR_TUNABLEOP", "1") != "0":
        assert torch.cuda.tunable.is_enabled()
    assert torch.equal(y, ref)
