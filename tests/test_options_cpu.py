"""CPU: kernel selection is a constructor argument (avr_amd.KernelOptions),
not process environment."""
import os
import re

import pytest
import torch

from avr_amd import KernelOptions
from avr_amd import options as O
from avr_amd.model import AVRModel, AVRModel_complex
from avr_amd.workloads import MESHRIR_MODEL, RAF_MODEL

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_package_reads_environment_only_in_options():
    """`os.environ` / getenv appear in avr_amd/*.py only inside options.py
    (KernelOptions.from_env for tools, and the two tuning knobs)."""
    hits = []
    pkg = os.path.join(ROOT, "avr_amd")
    for f in sorted(os.listdir(pkg)):
        if f.endswith(".py") and f != "options.py":
            text = open(os.path.join(pkg, f)).read()
            if re.search(r"os\.environ|getenv\(", text):
                hits.append(f)
    assert not hits, hits
    text = open(os.path.join(pkg, "options.py")).read()
    assert set(re.findall(r'"(AVR_[A-Z_]+)"', text)) == {"AVR_NSPLIT", "AVR_KSPLIT", "AVR_OPT_"}


def test_defaults_and_validation():
    o = KernelOptions()
    assert o.fused_sigma and o.fused_h1 and o.grouped_concat and o.fused_dgrad and o.out1 and o.tunableop
    assert o.narrow == "80" and o.hashgrid_bwd == "partitioned"
    with pytest.raises(ValueError):
        KernelOptions(narrow="1")
    with pytest.raises(ValueError):
        KernelOptions(hashgrid_bwd="sorted")
    with pytest.raises(TypeError):
        O.resolve({"narrow": "off"})


def test_from_env_is_explicit(monkeypatch):
    monkeypatch.setenv("AVR_OPT_FUSED_SIGMA", "0")
    monkeypatch.setenv("AVR_OPT_NARROW", "off")
    monkeypatch.setenv("AVR_OPT_WGRAD_MIN", "1024")
    # constructing a model does not read them ...
    m = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254))
    assert m.options == KernelOptions()
    # ... only an explicit from_env() does
    o = KernelOptions.from_env()
    assert (o.fused_sigma, o.narrow, o.wgrad_min, o.tunableop) == (False, "off", 1024, True)


def test_options_reach_every_submodule():
    o = KernelOptions(narrow="off", hashgrid_bwd="atomic")
    m = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=254), options=o)
    carriers = [s for s in m.modules() if hasattr(s, "options")]
    assert len(carriers) >= 1 + 3 + 6  # the model, its three MLPs, six hash grids
    assert all(s.options is o for s in carriers)
    o2 = KernelOptions(fused_sigma=False)
    O.apply(m, o2)
    assert all(s.options is o2 for s in carriers)


def test_backward_kernel_choice_is_recorded_in_forward():
    """_LinearReLU decides its data-gradient kernel in the forward: on the
    CPU (no HIP kernel applies) every layer records the GEMM path, and a
    masked chain applies the mask itself (no 512-wide kernel reached)."""
    from avr_amd import model as M

    torch.manual_seed(0)
    mlp = M.MLP(16, 8, {"n_neurons": 512, "n_hidden_layers": 3}, dtype=torch.float32)
    x = torch.randn(5, 16, requires_grad=True)
    ctxs = []
    orig = M._LinearReLU.forward

    def spy(ctx, *a):
        y = orig(ctx, *a)
        ctxs.append(ctx)
        return y

    M._LinearReLU.forward = staticmethod(spy)
    try:
        y = mlp(x)
        y.sum().backward()
    finally:
        M._LinearReLU.forward = staticmethod(orig)
    assert ctxs and all(c.dgrad == "gemm" for c in ctxs)
    ref = torch.nn.Sequential(*[torch.nn.Sequential(l, torch.nn.ReLU()) for l in mlp.layers[:-1]], mlp.layers[-1])
    x2 = x.detach().clone().requires_grad_(True)
    ref(x2).sum().backward()
    assert torch.allclose(x.grad, x2.grad, rtol=1e-5, atol=1e-6)
