"""The shipped TunableOp results for the width-512 hidden layers
(avr_amd/tunableop_gfx950.csv, avr_amd/model.py::_enable_tuned_gemms): file
format and the loader's guards on the CPU; on the GPU, the tuned solution's
output against the default hipBLASLt solution's, bit for bit, and the rule
that the drop-in leaves the caller's TunableOp state as it found it
(SURVEY.md §8(b) Ownership / Threading)."""
import csv
import os

import pytest
import torch

from avr_amd import model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_results_file_format():
    """Validators pin the libraries and gfx950; one entry per MLP dtype for
    the config-2 and config-5 inference shapes (M = 262,144 and 2,097,152
    rows, 512 -> 512)."""
    rows = list(csv.reader(open(model._TUNED_FILE)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    for k in ("PT_VERSION", "HIP_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION"):
        assert k in val
    ops = {(r[0], r[1]): r[2:] for r in rows if r[0] != "Validator"}
    assert len(ops) == 4
    for dt in ("Half", "BFloat16"):
        for m in (262144, 2097152):
            sol, ms = ops[(f"GemmAndBiasTunableOp_{dt}_TN", f"tn_512_{m}_512_ld_512_512_512")]
            assert sol.startswith("Gemm_") and float(ms) > 0


def test_tuned_shapes_parsed():
    """Only the file's own shapes take the TunableOp window."""
    assert model._TUNED_SHAPES == {(dt, m, 512, 512) for dt in (torch.float16, torch.bfloat16)
                                   for m in (262144, 2097152)}  # configs 2 and 5
    x = torch.empty(1000, 512, dtype=torch.float16)
    w = torch.empty(512, 512, dtype=torch.float16)
    assert not model._tuned_gemm(x, w)  # shape not in the file: no device call at all


def test_loader_respects_opt_out(monkeypatch):
    """AVR_TUNABLEOP=0 returns before touching TunableOp or the device (on
    this CPU-only container any such call would raise)."""
    monkeypatch.setattr(model, "_TUNED", [None])
    monkeypatch.setenv("AVR_TUNABLEOP", "0")
    assert model._enable_tuned_gemms(torch.device("cpu")) is False
    assert model._TUNED[0] is False


def _state():
    tun = torch.cuda.tunable
    return (tun.is_enabled(), tun.tuning_is_enabled(), tun.record_untuned_is_enabled(), tun.get_filename())


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [262144, 2097152], ids=["c2", "c5"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_tuned_layer_bit_identical(dtype, rows):
    """relu(x W^T) through _LinearReLU with the shipped solution equals the
    default hipBLASLt solution's output bit for bit (TunableOp off), with the
    tuned entry verifiably loaded, and TunableOp left as it was: config 2's
    262,144 rows and config 5's 2,097,152."""
    if os.environ.get("AVR_TUNABLEOP", "1") == "0":
        pytest.skip("AVR_TUNABLEOP=0: the shipped solution is switched off")
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.relu(torch.randn(rows, 512, device=dev, generator=g)).to(dtype)
    w = torch.randn(512, 512, device=dev, generator=g) / 512 ** 0.5
    bias = torch.zeros(512, dtype=dtype, device=dev)
    before = _state()
    assert not before[0]
    ref = torch._addmm_activation(bias, x, w.to(dtype).t(), use_gelu=False)
    assert model._enable_tuned_gemms(dev), "shipped TunableOp results rejected (validators?)"
    name = "Half" if dtype == torch.float16 else "BFloat16"
    res = {(r[0], r[1]): r[2] for r in torch.cuda.tunable.get_results()}
    assert res.get((f"GemmAndBiasTunableOp_{name}_TN", f"tn_512_{rows}_512_ld_512_512_512"), "").startswith(
        "Gemm_Hipblaslt_")
    assert model._tuned_gemm(x, w.to(dtype))
    with torch.no_grad():
        y = model._LinearReLU.apply(x, w, dtype)
    assert _state() == before
    assert torch.equal(y, ref)


@pytest.mark.gpu
def test_drop_in_leaves_tunableop_state():
    """AVRModel inference at the tuned shape (config 2, fp16 MLPs, the bench's
    network_inference) and a training step's forward + backward leave
    is_enabled / tuning / recording / filename as the caller had them."""
    from avr_amd import AVRRender, spectrum_to_ir
    from avr_amd.model import AVRModel
    from avr_amd.workloads import MESHRIR_MODEL, WORKLOADS

    dev = torch.device("cuda", 0)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    before = _state()
    torch.manual_seed(0)
    net = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=w.T), mlp_dtype=torch.float16).to(dev)
    r = AVRRender(net, **w.render)
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(1, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(1, 3, device=dev, generator=g) * 4 - 2
    with torch.no_grad():
        ir = spectrum_to_ir(r(ro, tx))
    torch.cuda.synchronize()
    assert torch.isfinite(ir).all()
    assert _state() == before
    out = r(ro, tx)
    out.abs().mean().backward()
    torch.cuda.synchronize()
    assert _state() == before
