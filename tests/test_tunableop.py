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
    rows, 512 -> 512), and the bf16 MLP GEMMs of the config-3 / -4 training
    steps (83,200 and 147,712 rows): forward (TN, with the ReLU epilogue) and
    data gradient (NN).  No "Default" rows (nothing to switch on for them)."""
    rows = list(csv.reader(open(model._TUNED_FILE)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    for k in ("PT_VERSION", "HIP_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION"):
        assert k in val
    ops = {(r[0], r[1]): r[2:] for r in rows if r[0] != "Validator"}
    assert len(ops) == len([r for r in rows if r[0] != "Validator"])  # no duplicates
    for dt in ("Half", "BFloat16"):
        for m in (262144, 2097152):
            sol, ms = ops[(f"GemmAndBiasTunableOp_{dt}_TN", f"tn_512_{m}_512_ld_512_512_512")]
            assert sol.startswith("Gemm_") and float(ms) > 0
    for (op, sig), (sol, ms) in ops.items():
        assert sol.startswith("Gemm_") and float(ms) > 0, (op, sig)
        if op.startswith("GemmTunableOp_"):
            assert op == "GemmTunableOp_BFloat16_NN" and int(sig.split("_")[2]) in (83200, 147712)
    assert ("GemmTunableOp_BFloat16_NN", "nn_80_83200_128_ld_80_128_80") in ops


def test_tuned_shapes_parsed():
    """Only the file's own shapes take the TunableOp window."""
    S = model._TUNED_SHAPES
    assert {("relu", dt, m, 512, 512) for dt in (torch.float16, torch.bfloat16)
            for m in (262144, 2097152)} <= S  # configs 2 and 5
    assert ("dgrad", torch.bfloat16, 83200, 128, 80) in S  # g [83200, 128] @ W [128, 80]
    assert ("relu", torch.bfloat16, 83200, 512, 416) in S
    assert all(k[0] in ("relu", "dgrad") for k in S)
    x = torch.empty(1000, 512, dtype=torch.float16)
    w = torch.empty(512, 512, dtype=torch.float16)
    assert not model._tuned_gemm(x, w)  # shape not in the file: no device call at all
    assert not model._tuned_dgrad(x, w)


def test_opt_out_never_touches_tunableop(monkeypatch):
    """KernelOptions(tunableop=False) returns before touching TunableOp or the
    device (on this CPU-only container any such call would raise)."""
    from avr_amd.options import KernelOptions

    monkeypatch.setattr(model, "_TUNED", [None])
    x = torch.empty(262144, 512, dtype=torch.float16)
    w = torch.empty(512, 512, dtype=torch.float16)
    off = KernelOptions(tunableop=False)
    assert not model._tuned_gemm(x, w, off)
    assert not model._tuned_dgrad(x, w, off)
    assert model._TUNED[0] is None


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
    assert len(res) >= 25
    assert res.get((f"GemmAndBiasTunableOp_{name}_TN", f"tn_512_{rows}_512_ld_512_512_512"), "").startswith(
        "Gemm_Hipblaslt_")
    assert model._tuned_gemm(x, w.to(dtype))
    with torch.no_grad():
        y = model._LinearReLU.apply(x, w, dtype)
    assert _state() == before
    assert torch.equal(y, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,out,inp", [(83200, 128, 80), (83200, 512, 416), (147712, 256, 128)])
def test_tuned_dgrad_bit_identical(rows, out, inp):
    """The data gradient g @ W through `_mm_dgrad` with the shipped solution
    equals the default solution's output bit for bit, and TunableOp is left
    as it was (config-3 / -4 training shapes)."""
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(rows + out)
    g = torch.randn(rows, out, device=dev, generator=gen).to(torch.bfloat16)
    w = (torch.randn(out, inp, device=dev, generator=gen) / out ** 0.5).to(torch.bfloat16)
    before = _state()
    ref = g @ w
    assert model._tuned_dgrad(g, w)
    gx = model._mm_dgrad(g, w)
    assert _state() == before
    assert torch.equal(gx, ref)


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
