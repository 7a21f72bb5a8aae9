"""State-dict interchange with the reference's tcnn modules
(avr_amd.tcnn_compat): tcnn's flat `params` of an MLP (weights row-major
[out][in] per layer, input and output widths padded to 16) round-trip
through our per-layer weights; whole-model state dicts convert both ways.
Parity unpinned: no reference checkpoint exists (tinycudann is absent)."""
import torch

from avr_amd.model import MLP, AVRModel, AVRModel_complex
from avr_amd.tcnn_compat import (from_reference, is_reference_layout, mlp_from_tcnn, mlp_to_tcnn,
                                 tcnn_n_params, to_reference)
from avr_amd.workloads import MESHRIR_MODEL, RAF_MODEL


def test_mlp_param_count_and_padding():
    # MeshRIR signal network (model.py:176-180): 208 -> 512 x3 -> 1022
    m = MLP(208, 1022, dict(n_neurons=512, n_hidden_layers=3))
    assert tcnn_n_params(m) == 512 * 208 + 2 * 512 * 512 + 1024 * 512
    # sigma decoder: 128 -> 1 (output padded to 16 rows), input 40 -> 48
    d = MLP(40, 1, dict(n_neurons=128, n_hidden_layers=1))
    assert tcnn_n_params(d) == 128 * 48 + 16 * 128
    flat = mlp_to_tcnn(d)
    w0 = flat[:128 * 48].view(128, 48)
    assert torch.equal(w0[:, :40], d.layers[0].weight.detach()) and not w0[:, 40:].any()
    last = flat[128 * 48:].view(16, 128)
    assert torch.equal(last[0], d.layers[1].weight.detach()[0]) and not last[1:].any()


def test_mlp_round_trip():
    torch.manual_seed(0)
    a = MLP(83, 7, dict(n_neurons=64, n_hidden_layers=2))
    b = MLP(83, 7, dict(n_neurons=64, n_hidden_layers=2))
    mlp_from_tcnn(b, mlp_to_tcnn(a))
    for la, lb in zip(a.layers, b.layers):
        assert torch.equal(la.weight, lb.weight)


def test_model_state_dict_round_trip():
    torch.manual_seed(1)
    for cls, cfg in ((AVRModel, dict(MESHRIR_MODEL, signal_output_dim=254)),
                     (AVRModel_complex, dict(RAF_MODEL, signal_output_dim=254))):
        src, dst = cls(cfg), cls(cfg)
        ref_sd = to_reference(src)
        assert is_reference_layout(dst, ref_sd) and not is_reference_layout(dst, src.state_dict())
        assert any(k.endswith("_model_signal.params") for k in ref_sd)
        assert not any(".layers." in k for k in ref_sd)
        from_reference(dst, ref_sd)
        for (k, v), (k2, v2) in zip(src.state_dict().items(), dst.state_dict().items()):
            assert k == k2 and torch.equal(v, v2), k


def _reference_param_list(model):
    """The reference module's parameters in its order (model.py:66-180,
    258-289): one flat tensor per tcnn Encoding / Network."""
    ref_sd = to_reference(model)
    order = [n for n, _ in model.named_parameters()]
    flat, seen = [], set()
    for name in order:
        key = name if not ".layers." in name else name.split(".layers.")[0] + ".params"
        if key not in seen:
            seen.add(key)
            flat.append(torch.nn.Parameter(ref_sd[key].clone()))
    return flat


def test_adam_state_to_reference_loads_into_flat_optimizer():
    """The Adam state a reference-layout checkpoint carries loads into an
    optimizer built over the reference's flat per-module parameters (what
    avr_runner.py:121-124 does after loading the weights), and converts
    back to the same per-layer state."""
    from avr_amd.tcnn_compat import optimizer_state_from_reference, optimizer_state_to_reference, param_units

    torch.manual_seed(3)
    for cls, cfg in ((AVRModel, dict(MESHRIR_MODEL, signal_output_dim=254)),
                     (AVRModel_complex, dict(RAF_MODEL, signal_output_dim=254))):
        model = cls(cfg)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        for p in model.parameters():
            p.grad = torch.randn_like(p) * 1e-3
        opt.step()
        opt.step()
        ref_state = optimizer_state_to_reference(model, opt.state_dict())
        flat = _reference_param_list(model)
        assert len(param_units(model)) == len(flat)
        ref_opt = torch.optim.Adam(flat, lr=1e-3)
        ref_opt.load_state_dict(ref_state)  # the reference's call: must not raise
        for j, p in enumerate(flat):
            st = ref_opt.state[p]
            assert st["exp_avg"].shape == p.shape and float(st["step"]) == 2.0
        back = optimizer_state_from_reference(model, ref_opt.state_dict(), opt.state_dict()["param_groups"])
        opt2 = torch.optim.Adam(model.parameters(), lr=1e-3)
        opt2.load_state_dict(back)
        for p in model.parameters():
            a, b = opt.state[p], opt2.state[p]
            assert torch.equal(a["exp_avg"], b["exp_avg"]) and torch.equal(a["exp_avg_sq"], b["exp_avg_sq"])
            assert float(a["step"]) == float(b["step"])


def test_adam_state_from_reference_rejects_mismatch():
    """A reference optimizer state over another parameter count raises
    ValueError (TrainStep.load_checkpoint then restarts the optimiser)."""
    import pytest

    from avr_amd.tcnn_compat import optimizer_state_from_reference, optimizer_state_to_reference

    model = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=254))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    ref_state = optimizer_state_to_reference(model, opt.state_dict())
    ref_state["param_groups"][0]["params"] = ref_state["param_groups"][0]["params"][:-1]
    with pytest.raises(ValueError):
        optimizer_state_from_reference(model, ref_state, opt.state_dict()["param_groups"])
