"""GPU: the training-loop body (avr_amd/training.py, avr_runner.py:160-200):
gradient clip + NaN/Inf zeroing kernel against torch's ops, a full
TrainStep with the HIP criterion, and the checkpoint round trip."""
import pytest
import torch

from avr_amd import AVRRender
from avr_amd.model import AVRModel_complex
from avr_amd.training import TrainStep, clip_and_sanitize_
from avr_amd.workloads import RAF, RAF_MODEL

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

RAF_TRAIN = dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5,
                 spec_loss_weight=1, amplitude_loss_weight=1, angle_loss_weight=1,
                 time_loss_weight=20, energy_loss_weight=3, multistft_loss_weight=2)


def _params(seed, poison):
    g = torch.Generator(device=DEV).manual_seed(seed)
    shapes = [(1000,), (37, 13), (4096, 2), (7,), (300001,)]
    ps = []
    for i, s in enumerate(shapes):
        p = torch.nn.Parameter(torch.zeros(s, device=DEV))
        p.grad = torch.randn(s, device=DEV, generator=g) * (3.0 if i == 2 else 0.5)
        ps.append(p)
    if poison:
        ps[1].grad.view(-1)[5] = float("nan")
        ps[4].grad[17] = float("inf")
        ps[4].grad[99] = -float("inf")
    return ps


@pytest.mark.parametrize("poison", [False, True])
def test_clip_and_sanitize_matches_reference_ops(poison):
    a = _params(0, poison)
    b = _params(0, poison)
    torch.nn.utils.clip_grad_norm_(a, max_norm=1)
    for p in a:  # avr_runner.py:192-196
        p.grad[p.grad != p.grad] = 0
        p.grad[torch.isinf(p.grad)] = 0
    clip_and_sanitize_(b, max_norm=1)
    for pa, pb in zip(a, b):
        assert torch.equal(pa.grad, pb.grad)


def test_clip_leaves_small_gradients_unscaled():
    ps = _params(1, False)
    for p in ps:
        p.grad.mul_(1e-4)
    ref = [p.grad.clone() for p in ps]
    clip_and_sanitize_(ps, max_norm=1)
    for p, r in zip(ps, ref):
        assert torch.equal(p.grad, r)


def _setup(seed=0):
    torch.manual_seed(seed)
    cfg = dict(RAF, n_azi=8, n_ele=4, n_samples=16)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800)).to(DEV)
    r = AVRRender(model, **cfg).to(DEV)
    B = 2
    g = torch.Generator(device=DEV).manual_seed(7)
    rx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
    t = torch.arange(800, device=DEV)
    ir = torch.randn(B, 800, device=DEV, generator=g) * torch.exp(-t / 120.0) * 0.05
    ori = torch.fft.rfft(ir)
    return r, ori, rx, tx, dtx


def test_train_step_reduces_loss_and_updates_all_parameters():
    r, ori, rx, tx, dtx = _setup()
    step = TrainStep(r, RAF_TRAIN, dict(fs=16000, speed=346.8))
    before = {n: p.detach().clone() for n, p in r.named_parameters()}
    totals = []
    for _ in range(8):
        torch.manual_seed(1)  # same ray jitter each step
        total, losses = step(ori, rx, tx, dtx)
        totals.append(float(total))
        assert all(torch.isfinite(x) for x in losses)
    assert totals[-1] < totals[0], totals
    changed = [n for n, p in r.named_parameters() if not torch.equal(p.detach(), before[n])]
    assert len(changed) == len(before), set(before) - set(changed)
    assert step.current_iteration == 8
    # CosineAnnealingLR stepped once per iteration
    assert step.optimizer.param_groups[0]["lr"] < 2e-4


def test_checkpoint_round_trip(tmp_path):
    r, ori, rx, tx, dtx = _setup()
    step = TrainStep(r, RAF_TRAIN, dict(fs=16000, speed=346.8))
    for _ in range(3):
        torch.manual_seed(1)
        step(ori, rx, tx, dtx)
    path = step.save_checkpoint(str(tmp_path / "000003.tar"))
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"current_iteration", "audionerf_network_state_dict",
                       "optimizer_state_dict", "scheduler_state_dict"}
    assert all(k.startswith("network_fn.") for k in ck["audionerf_network_state_dict"])
    torch.manual_seed(1)
    ref_total, _ = step(ori, rx, tx, dtx)

    r2, _, _, _, _ = _setup(seed=123)  # different init, then restored
    step2 = TrainStep(r2, RAF_TRAIN, dict(fs=16000, speed=346.8))
    step2.load_checkpoint(path)
    assert step2.current_iteration == 3
    torch.manual_seed(1)
    total2, _ = step2(ori, rx, tx, dtx)
    assert abs(float(total2) - float(ref_total)) <= 1e-6 * abs(float(ref_total))


@pytest.mark.gpu
def test_checkpoint_reference_layout(tmp_path):
    """A checkpoint whose networks are tcnn flat `params` (the reference's
    modules, avr_amd.tcnn_compat) restores the same weights: written by
    save_checkpoint(reference_layout=True) it resumes exactly; with the
    reference's flat-parameter Adam state the weights and the state load
    (converted per layer); a state over another parameter count restarts
    the optimiser with a warning."""
    r, ori, rx, tx, dtx = _setup()
    step = TrainStep(r, RAF_TRAIN, dict(fs=16000, speed=346.8))
    for _ in range(2):
        torch.manual_seed(1)
        step(ori, rx, tx, dtx)
    path = step.save_checkpoint(str(tmp_path / "ref.tar"), reference_layout=True)
    sd = torch.load(path, weights_only=True)["audionerf_network_state_dict"]
    assert any(k.endswith("_model_signal.params") for k in sd) and not any(".layers." in k for k in sd)
    torch.manual_seed(1)
    ref_total, _ = step(ori, rx, tx, dtx)

    r2, _, _, _, _ = _setup(seed=123)
    step2 = TrainStep(r2, RAF_TRAIN, dict(fs=16000, speed=346.8))
    step2.load_checkpoint(path)
    torch.manual_seed(1)
    total2, _ = step2(ori, rx, tx, dtx)
    assert abs(float(total2) - float(ref_total)) <= 1e-6 * abs(float(ref_total))

    # the reference's own optimiser state: one moment tensor per flat params,
    # in the reference's module order (the order of the `.params` keys)
    ck = torch.load(path, weights_only=True)
    flat = [v for k, v in ck["audionerf_network_state_dict"].items() if k.endswith(".params")]
    ck["optimizer_state_dict"]["state"] = {
        i: {"step": torch.tensor(2.0), "exp_avg": torch.full_like(v, 1e-3), "exp_avg_sq": torch.zeros_like(v)}
        for i, v in enumerate(flat)}
    ck["optimizer_state_dict"]["param_groups"][0]["params"] = list(range(len(flat)))
    torch.save(ck, str(tmp_path / "ref_opt.tar"))
    r3, _, _, _, _ = _setup(seed=321)
    step3 = TrainStep(r3, RAF_TRAIN, dict(fs=16000, speed=346.8))
    step3.load_checkpoint(str(tmp_path / "ref_opt.tar"))  # converted, no warning
    from avr_amd.tcnn_compat import to_reference
    got = to_reference(r3)
    for k, v in ck["audionerf_network_state_dict"].items():
        assert torch.equal(got[k].cpu(), v.cpu()), k
    for p in r3.parameters():
        st = step3.optimizer.state[p]
        assert float(st["step"]) == 2.0 and st["exp_avg"].shape == p.shape
        assert torch.all(st["exp_avg"] == 1e-3)
    # a state over another parameter count: weights load, the optimiser restarts
    ck["optimizer_state_dict"]["param_groups"][0]["params"] = list(range(len(flat) - 1))
    ck["optimizer_state_dict"]["state"].pop(len(flat) - 1)
    torch.save(ck, str(tmp_path / "ref_opt_bad.tar"))
    r4, _, _, _, _ = _setup(seed=322)
    step4 = TrainStep(r4, RAF_TRAIN, dict(fs=16000, speed=346.8))
    with pytest.warns(RuntimeWarning, match="optimizer state not restored"):
        step4.load_checkpoint(str(tmp_path / "ref_opt_bad.tar"))
    assert not step4.optimizer.state


@pytest.mark.gpu
@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_native_adam_matches_torch_adam(wd):
    """clip_sanitize_adam_ (avr_adam_step) against clip_and_sanitize_ +
    torch.optim.Adam over 5 steps, including poisoned (NaN/Inf) gradients and
    a parameter without a gradient; state_dict layouts interchangeable."""
    from avr_amd.training import clip_sanitize_adam_
    g = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(1000, 3), (7,), (4096, 2), (5, 5)]
    ref = [torch.randn(s, device=DEV, generator=g).requires_grad_(True) for s in shapes]
    mine = [p.detach().clone().requires_grad_(True) for p in ref]
    o_ref = torch.optim.Adam(ref, lr=1e-3, betas=(0.9, 0.999), weight_decay=wd)
    o_mine = torch.optim.Adam(mine, lr=1e-3, betas=(0.9, 0.999), weight_decay=wd)
    for it in range(5):
        for k, (a, b) in enumerate(zip(ref, mine)):
            if k == 3 and it < 2:  # no gradient for the first two steps
                a.grad = b.grad = None
                continue
            gr = torch.randn(a.shape, device=DEV, generator=g) * (3.0 if it % 2 else 0.1)
            if k == 0:
                gr.view(-1)[::97] = float("nan")
                gr.view(-1)[5] = float("inf")
            a.grad, b.grad = gr.clone(), gr.clone()
        clip_and_sanitize_(ref, max_norm=1)
        o_ref.step()
        clip_sanitize_adam_(o_mine, max_norm=1)
        for a, b in zip(ref, mine):
            torch.testing.assert_close(b.detach(), a.detach(), rtol=2e-6, atol=2e-7)
    for a, b in zip(ref, mine):
        sa, sb = o_ref.state[a], o_mine.state[b]
        assert float(sa["step"]) == float(sb["step"]) and not sb["step"].is_cuda
        torch.testing.assert_close(sb["exp_avg"], sa["exp_avg"], rtol=2e-6, atol=1e-9)
        torch.testing.assert_close(sb["exp_avg_sq"], sa["exp_avg_sq"], rtol=2e-6, atol=1e-12)


@pytest.mark.gpu
def test_native_adam_invalidates_inference_caches():
    """The one-pass Adam bumps the parameters' version counters, so weight
    casts cached at inference (wcache.cast_weight) are rebuilt after a step."""
    from avr_amd.training import clip_sanitize_adam_
    from avr_amd.wcache import cast_weight
    p = torch.nn.Parameter(torch.randn(64, 32, device=DEV))
    opt = torch.optim.Adam([p], lr=1e-2)
    with torch.no_grad():
        c0 = cast_weight(p, torch.bfloat16, True).clone()
    p.grad = torch.randn_like(p)
    v0 = p._version
    clip_sanitize_adam_(opt, max_norm=1)
    assert p._version > v0
    with torch.no_grad():
        c1 = cast_weight(p, torch.bfloat16, True)
    torch.testing.assert_close(c1, p.detach().to(torch.bfloat16), rtol=0, atol=0)
    assert not torch.equal(c1, c0)


@pytest.mark.gpu
def test_native_adam_many_tensors_and_empty():
    """More tensors than one kernel-argument table holds (32), an empty one,
    odd sizes (scalar tail), against clip_and_sanitize_ + torch Adam."""
    from avr_amd.training import clip_sanitize_adam_
    g = torch.Generator(device=DEV).manual_seed(9)
    shapes = [(0,)] + [(37 + 5 * k,) for k in range(40)] + [(3, 7)]
    ref = [torch.randn(s, device=DEV, generator=g).requires_grad_(True) for s in shapes]
    mine = [p.detach().clone().requires_grad_(True) for p in ref]
    o_ref = torch.optim.Adam(ref, lr=3e-3)
    o_mine = torch.optim.Adam(mine, lr=3e-3)
    for _ in range(3):
        for a, b in zip(ref, mine):
            gr = torch.randn(a.shape, device=DEV, generator=g)
            a.grad, b.grad = gr.clone(), gr.clone()
        clip_and_sanitize_(ref, max_norm=1)
        o_ref.step()
        clip_sanitize_adam_(o_mine, max_norm=1)
    for a, b in zip(ref, mine):
        torch.testing.assert_close(b.detach(), a.detach(), rtol=2e-6, atol=2e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["plain", "small", "nan", "inf", "many", "empty"])
def test_native_clip_coef_matches_torch_norm(case):
    """avr_grad_clip_coef (the fused Adam path's clip coefficient) against
    torch's foreach norm: equal within fp32 rounding, NaN / Inf propagated as
    torch does, identical from run to run (fixed summation order)."""
    from avr_amd.training import _clip_coef, _native_clip_coef
    g = torch.Generator(device=DEV).manual_seed(11)
    shapes = {"many": [(s,) for s in range(1, 70)] + [(1 << 20,)], "empty": [(0,), (5,)]}.get(
        case, [(1 << 21,), (7,), (512, 512), (3, 1000), (1 << 18, 2)])
    grads = [torch.randn(s, device=DEV, generator=g) * (1e-4 if case == "small" else 0.5) for s in shapes]
    if case == "nan":
        grads[2].view(-1)[12345] = float("nan")
    if case == "inf":
        grads[0].view(-1)[77] = -float("inf")
    t_ref, c_ref = _clip_coef(grads, 1.0)
    t0, c0 = _native_clip_coef(grads, 1.0, DEV)
    t1, c1 = _native_clip_coef(grads, 1.0, DEV)
    torch.cuda.synchronize()
    bits = lambda t: t.view(torch.int32)  # noqa: E731  (NaN == NaN bit for bit)
    assert torch.equal(bits(t0), bits(t1)) and torch.equal(bits(c0), bits(c1))
    if case == "nan":
        assert torch.isnan(t0) and torch.isnan(c0) and torch.isnan(c_ref)
    elif case == "inf":
        assert torch.isinf(t0) and float(c0) == 0.0 == float(c_ref)
    else:
        torch.testing.assert_close(t0, t_ref.float(), rtol=1e-5, atol=0)
        torch.testing.assert_close(c0, c_ref.float(), rtol=1e-5, atol=0)
        if case == "small":
            assert float(c0) == 1.0
