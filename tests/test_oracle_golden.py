"""CPU: the oracle (oracle/avr_oracle.py) against golden vectors produced by
the real reference renderer_cpu.py (tools/gen_golden.py)."""
import numpy as np
import pytest
import torch

from golden_util import Case, case_names, digest_check, rel_l2
from oracle import avr_oracle as orc

CASES = case_names()
FAST = [c for c in CASES if not c.startswith(("c2", "c5", "c4"))]


def _run(case, record=None, grads=False):
    inp = case.inputs()
    w = case.workload
    attn = torch.from_numpy(inp["attn"]).requires_grad_(grads)
    sig = torch.from_numpy(inp["signal"]).requires_grad_(grads)
    dtx = None if inp["direction_tx"] is None else torch.from_numpy(inp["direction_tx"])
    torch.manual_seed(case.seed)
    out = orc.render_spectrum(orc.RenderConfig.from_kwargs(**w.render), orc.StubNetwork(attn, sig),
                              torch.from_numpy(inp["rays_o"]), torch.from_numpy(inp["position_tx"]),
                              dtx, record=record)
    return out, attn, sig


def test_fixtures_present():
    assert len(CASES) >= 9, CASES


@pytest.mark.parametrize("name", CASES)
def test_oracle_forward_matches_reference(name):
    case = Case(name)
    rec = {}
    out, _, _ = _run(case, rec)
    ref = case["out"]
    o = out.numpy()
    rel = rel_l2(o, ref)
    # bit-identical where generated; allow libm/thread-order noise elsewhere
    assert rel < 1e-6, rel
    np.testing.assert_allclose(rec["u_azi"].numpy(), case["u_azi"], rtol=0, atol=0)
    np.testing.assert_allclose(rec["dirs"].numpy(), case["dirs"], rtol=0, atol=2e-7)
    np.testing.assert_array_equal(rec["shift"].numpy(), case["shift"])
    digest_check(case, "weights", rec["weights"].numpy(), rtol=1e-5, atol=1e-9)
    # integer work is bit-exact: every delay of every fixture
    np.testing.assert_array_equal(rec["delay"].numpy().astype(np.int16), case["delay"])
    for k in ("pts", "view", "tx", "dir_tx"):
        if case.has("net_" + k + "_sum"):
            digest_check(case, "net_" + k, rec[k].numpy(), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", CASES)
def test_oracle_ir_matches_reference(name):
    case = Case(name)
    ir = orc.spectrum_to_ir(torch.from_numpy(case["out"])).numpy()
    np.testing.assert_allclose(ir, case["ir"], rtol=1e-5, atol=1e-6 * np.abs(case["ir"]).max())


@pytest.mark.parametrize("name", [c for c in FAST if Case(c).grads])
def test_oracle_backward_matches_reference(name):
    case = Case(name)
    out, attn, sig = _run(case, grads=True)
    (out * torch.from_numpy(case.grad_probe())).sum().backward()
    ga = attn.grad.float().numpy()
    gs = sig.grad.float().numpy()
    scale_a = np.sqrt(float(case["grad_attn_sumsq"]) / ga.size)
    scale_s = np.sqrt(float(case["grad_signal_sumsq"]) / gs.size)
    digest_check(case, "grad_attn", ga, rtol=1e-5, atol=1e-5 * scale_a)
    digest_check(case, "grad_signal", gs, rtol=1e-5, atol=1e-5 * scale_s)
