"""GPU parity: the HIP render path against the golden vectors of the real
reference and against the CPU oracle on the same seeded inputs.

Tolerance (BASELINE.json north_star): 1e-4 relative on the rendered complex
spectrum (L2 and max-norm).  Integer delays: bit-exact on every entry of
every fixture, both from the kernel's own ray directions and from the
reference's directions fed in."""
import ctypes

import numpy as np
import pytest
import torch

from golden_util import Case, case_names, digest_check, rel_l2, rel_max
from oracle import avr_oracle as orc

from avr_amd import AVRRender, spectrum_to_ir
from avr_amd import _lib
from avr_amd.renderer import get_tables, render_params
from avr_amd.workloads import WORKLOADS, make_inputs

pytestmark = pytest.mark.gpu
CASES = case_names()
TOL = 1e-4
DEV = torch.device("cuda", 0)


class Net(torch.nn.Module):
    """Stub network returning device tensors; records its inputs."""

    def __init__(self, attn, signal):
        super().__init__()
        self.attn, self.signal, self.seen = attn, signal, None

    def forward(self, pts, view, tx, dir_tx=None):
        self.seen = (pts, view, tx, dir_tx)
        return self.attn, self.signal


def hip_render(case_or_w, inp, seed, grads=False):
    w = case_or_w.workload if isinstance(case_or_w, Case) else case_or_w
    attn = torch.from_numpy(inp["attn"]).to(DEV).requires_grad_(grads)
    sig = torch.from_numpy(inp["signal"]).to(DEV).requires_grad_(grads)
    net = Net(attn, sig)
    r = AVRRender(net, **w.render)
    dtx = None if inp["direction_tx"] is None else torch.from_numpy(inp["direction_tx"]).to(DEV)
    torch.manual_seed(seed)
    out = r(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV), dtx)
    return out, attn, sig, net


@pytest.mark.parametrize("name", CASES)
def test_spectrum_matches_reference_golden(name):
    case = Case(name)
    out, *_ = hip_render(case, case.inputs(), case.seed)
    o = out.detach().cpu().numpy()
    ref = case["out"]
    assert rel_l2(o, ref) < TOL, rel_l2(o, ref)
    assert rel_max(o, ref) < TOL, rel_max(o, ref)


@pytest.mark.parametrize("name", CASES)
def test_ir_matches_reference_golden(name):
    case = Case(name)
    out, *_ = hip_render(case, case.inputs(), case.seed)
    ir = spectrum_to_ir(out.detach()).cpu().numpy()
    assert rel_l2(ir, case["ir"]) < TOL
    # the HIP irfft itself, on the reference spectrum
    ir2 = spectrum_to_ir(torch.from_numpy(case["out"]).to(DEV)).cpu().numpy()
    assert rel_l2(ir2, case["ir"]) < 1e-5


@pytest.mark.parametrize("name", CASES)
def test_network_inputs_and_directions(name):
    case = Case(name)
    inp = case.inputs()
    out, _, _, net = hip_render(case, inp, case.seed)
    for k, t in zip(("pts", "view", "tx", "dir_tx"), net.seen):
        if t is None:
            assert not case.has("net_" + k + "_sum")
            continue
        digest_check(case, "net_" + k, t.cpu().numpy(), rtol=0, atol=3e-6)


def _stage_weights(case, inp, ref_dirs=False):
    """Run ray generation + weights kernel; return (w, delay) as numpy.

    With ref_dirs the reference's own direction table (the fixture's `dirs`,
    torch-CPU trig) replaces the kernel-generated one, isolating the integer
    delay geometry (renderer_cpu.py:76-80) from the trig library."""
    w = case.workload
    r = AVRRender(None, **w.render)
    torch.manual_seed(case.seed)
    dtx = None if inp["direction_tx"] is None else torch.from_numpy(inp["direction_tx"]).to(DEV)
    _, _, _, _, geom = r.sample(torch.from_numpy(inp["rays_o"]).to(DEV),
                                torch.from_numpy(inp["position_tx"]).to(DEV), dtx)
    p = render_params(w.render, w.T)
    tables = get_tables(p, DEV)
    B, R, S = w.batch, w.n_rays, w.n_samples
    attn = torch.from_numpy(inp["attn"]).to(DEV).reshape(B, -1).contiguous()
    if ref_dirs:
        geom["dirs"] = torch.from_numpy(case["dirs"]).to(DEV).contiguous()
    wt = torch.empty(B, R, S, device=DEV)
    dl = torch.empty(B, R, S, dtype=torch.int32, device=DEV)
    _lib.call("avr_weights_fwd", ctypes.byref(p), B, attn.data_ptr(),
              0 if attn.dtype == torch.float32 else 1, geom["rays_o"].data_ptr(),
              geom["position_tx"].data_ptr(), geom["dirs"].data_ptr(), tables.d_vals.data_ptr(),
              wt.data_ptr(), dl.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return wt.cpu().numpy(), dl.cpu().numpy(), geom["dirs"].cpu().numpy(), tables


@pytest.mark.parametrize("name", CASES)
def test_stage_weights_delays_tables(name):
    case = Case(name)
    inp = case.inputs()
    wt, dl, dirs, tables = _stage_weights(case, inp)
    np.testing.assert_allclose(dirs, case["dirs"], rtol=0, atol=5e-7)
    np.testing.assert_allclose(tables.d_vals.cpu().numpy(), case["d_vals"], rtol=0, atol=0)
    np.testing.assert_array_equal(tables.shift.cpu().numpy(), case["shift"].astype(np.int32))
    # weights are <= 1; device expf and the tree-ordered transmittance scan
    # differ from torch's SLEEF expf + sequential cumprod by a few ulp
    digest_check(case, "weights", wt, rtol=1e-5, atol=2e-7)
    # integer delays: bit-exact, every entry (the fixtures hold them in full)
    np.testing.assert_array_equal(dl.astype(np.int16), case["delay"])


@pytest.mark.parametrize("name", CASES)
def test_delays_bit_exact_from_reference_directions(name):
    case = Case(name)
    wt, dl, _, _ = _stage_weights(case, case.inputs(), ref_dirs=True)
    np.testing.assert_array_equal(dl.astype(np.int16), case["delay"])
    digest_check(case, "weights", wt, rtol=1e-5, atol=2e-7)


@pytest.mark.parametrize("name", [c for c in CASES if Case(c).grads])
def test_backward_matches_reference_golden(name):
    case = Case(name)
    out, attn, sig, _ = hip_render(case, case.inputs(), case.seed, grads=True)
    g = torch.from_numpy(case.grad_probe()).to(DEV)
    (out * g).sum().backward()
    ga = attn.grad.float().cpu().numpy()
    gs = sig.grad.float().cpu().numpy()
    # relative to the gradient's RMS
    scale_a = np.sqrt(float(case["grad_attn_sumsq"]) / ga.size)
    scale_s = np.sqrt(float(case["grad_signal_sumsq"]) / gs.size)
    fp16 = case.workload.signal_dtype == "float16"
    tol_s = 2e-3 if fp16 else TOL  # fp16 gradient storage rounds at 2^-11
    digest_check(case, "grad_attn", ga, rtol=0, atol=TOL * 50 * scale_a + 1e-4 * np.abs(ga).max())
    digest_check(case, "grad_signal", gs, rtol=tol_s, atol=tol_s * scale_s)
    s64 = gs.astype(np.float64).sum()
    assert abs(s64 - float(case["grad_signal_sum"])) <= 1e-3 * np.sqrt(float(case["grad_signal_sumsq"]) * gs.size) + 1e-6
    dot = float((gs.astype(np.float64) * case.inputs()["signal"].astype(np.float64)).sum())
    ref_dot = float(case["grad_signal_dot_signal"])
    assert abs(dot - ref_dot) <= 1e-3 * abs(ref_dot) + 1e-6


@pytest.mark.parametrize("name", ["c1_s0", "edge_ragged_s3", "edge_oddT_s4", "c3_s0"])
def test_matches_oracle_same_seed(name):
    case = Case(name)
    inp = case.inputs()
    w = case.workload
    torch.manual_seed(case.seed)
    dtx = None if inp["direction_tx"] is None else torch.from_numpy(inp["direction_tx"])
    ref = orc.render_spectrum(orc.RenderConfig.from_kwargs(**w.render),
                              orc.StubNetwork(torch.from_numpy(inp["attn"]), torch.from_numpy(inp["signal"])),
                              torch.from_numpy(inp["rays_o"]), torch.from_numpy(inp["position_tx"]), dtx).numpy()
    out, *_ = hip_render(case, inp, case.seed)
    assert rel_l2(out.detach().cpu().numpy(), ref) < TOL


def test_deterministic_bitwise():
    case = Case("c3_s0")
    inp = case.inputs()
    a, *_ = hip_render(case, inp, 0)
    b, *_ = hip_render(case, inp, 0)
    assert torch.equal(a, b)


def test_unaligned_signal_uses_scalar_path():
    case = Case("c1_s1")
    inp = case.inputs()
    w = case.workload
    big = torch.zeros(inp["signal"].size + 1, dtype=torch.float32, device=DEV)
    sig = big[1:].view(inp["signal"].shape)  # 4-byte offset: not 16-byte aligned
    sig.copy_(torch.from_numpy(inp["signal"]))
    attn = torch.from_numpy(inp["attn"]).to(DEV)
    r = AVRRender(Net(attn, sig), **w.render)
    torch.manual_seed(case.seed)
    out = r(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV))
    assert rel_l2(out.cpu().numpy(), case["out"]) < TOL


def test_ch_idx_passthrough_rules():
    case = Case("c1_s1")
    inp = case.inputs()
    attn = torch.from_numpy(inp["attn"]).to(DEV)
    sig = torch.from_numpy(inp["signal"]).to(DEV)

    class WithCh(torch.nn.Module):
        def forward(self, pts, view, tx, ch_idx=None):
            self.ch = ch_idx
            return attn, sig

    class NoCh(torch.nn.Module):
        def forward(self, pts, view, tx):
            return attn, sig

    ro = torch.from_numpy(inp["rays_o"]).to(DEV)
    tx = torch.from_numpy(inp["position_tx"]).to(DEV)
    net = WithCh()
    AVRRender(net, **case.workload.render)(ro, tx, ch_idx=torch.tensor([3], device=DEV))
    assert int(net.ch[0]) == 3
    AVRRender(NoCh(), **case.workload.render)(ro, tx)  # no ch_idx keyword passed


def test_config_guard_like_reference():
    w = WORKLOADS["c1_meshrir_plumbing"].replace(far=40.0)  # shift > 1.5T
    inp = make_inputs(w, 0)
    with pytest.raises(RuntimeError, match="stack expects"):
        hip_render(w, inp, 0)


# ------------------------------------------------------------------ full size
def test_config2_full_size_properties():
    """Config 2 (headline workload): linearity in the signal, additivity over
    ray halves, and agreement with the golden spectrum."""
    case = Case("c2_s0")
    inp = case.inputs()
    w = case.workload
    out, *_ = hip_render(case, inp, case.seed)
    base = out.detach().cpu().numpy()
    assert rel_l2(base, case["out"]) < TOL
    inp2 = dict(inp)
    inp2["signal"] = inp["signal"] * np.float32(2.0)
    out2, *_ = hip_render(case, inp2, case.seed)
    np.testing.assert_allclose(out2.detach().cpu().numpy(), 2 * base, rtol=0, atol=1e-6 * np.abs(base).max())
    # zero the second half of the rays: spectrum(first) + spectrum(second) == base
    R, S, T = w.n_rays, w.n_samples, w.T
    half = R // 2
    a = inp["signal"].reshape(1, R, S, T).copy()
    b = a.copy()
    a[:, half:] = 0
    b[:, :half] = 0
    ia, ib = dict(inp), dict(inp)
    ia["signal"], ib["signal"] = a.reshape(inp["signal"].shape), b.reshape(inp["signal"].shape)
    oa, *_ = hip_render(case, ia, case.seed)
    ob, *_ = hip_render(case, ib, case.seed)
    s = oa.detach().cpu().numpy() + ob.detach().cpu().numpy()
    assert rel_l2(s, base) < 1e-5


def test_config5_full_size_properties():
    """Config 5 at full size (4096 rays x 512 samples x T=4094, fp16 storage,
    17.2 GB of signal): exact linearity (doubling fp16 inputs doubles every
    product and sum exactly), additivity over 4 ray shards (the multi-GPU
    decomposition), finite IR.  Golden parity at T=4094 is c5small's."""
    from avr_amd.parallel import shard_range

    w = WORKLOADS["c5_simu_4096x512x2048"]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(5)
    attn = (torch.rand(B, R * S, 1, device=DEV, generator=g) * 2).to(torch.float16)
    sig = torch.randn(B, R * S, T, device=DEV, generator=g, dtype=torch.float16) * 0.1
    ro = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    r = AVRRender(Net(attn, sig), **w.render)
    with torch.no_grad():
        torch.manual_seed(0)
        out, ir = r.render_ir(ro, tx)
        assert torch.isfinite(out).all() and torch.isfinite(ir).all() and float(out.abs().max()) > 0
        sig.mul_(2)
        torch.manual_seed(0)
        out2 = r(ro, tx)
        sig.mul_(0.5)
        torch.testing.assert_close(out2, 2 * out, rtol=0, atol=1e-7 * float(out.abs().max()))
        total = None
        for k in range(4):
            r0, r1 = shard_range(R, k, 4)
            rk = AVRRender(Net(attn[:, r0 * S:r1 * S], sig[:, r0 * S:r1 * S]), **w.render)
            rk.ray_range = (r0, r1)
            torch.manual_seed(0)
            part = rk(ro, tx)
            total = part if total is None else total + part
    assert rel_l2(total.cpu().numpy(), out.cpu().numpy()) < 1e-5
    del sig, attn
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n_shards", [2, 3])
def test_ray_range_shards_sum_to_full(n_shards):
    """Rays split into contiguous ranges (the multi-GPU ray sharding) sum to
    the single-device spectrum."""
    from avr_amd.parallel import shard_range

    case = Case("c3_s0")
    inp = case.inputs()
    w = case.workload
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    attn = torch.from_numpy(inp["attn"]).to(DEV).view(B, R, S, 1)
    sig = torch.from_numpy(inp["signal"]).to(DEV).view(B, R, S, T)
    ro = torch.from_numpy(inp["rays_o"]).to(DEV)
    tx = torch.from_numpy(inp["position_tx"]).to(DEV)
    dtx = torch.from_numpy(inp["direction_tx"]).to(DEV)
    total = None
    for k in range(n_shards):
        r0, r1 = shard_range(R, k, n_shards)
        net = Net(attn[:, r0:r1].reshape(B, -1, 1).contiguous(), sig[:, r0:r1].reshape(B, -1, T).contiguous())
        r = AVRRender(net, **w.render)
        r.ray_range = (r0, r1)
        torch.manual_seed(case.seed)
        part = r(ro, tx, dtx)
        assert net.seen[0].shape[1] == (r1 - r0) * S
        total = part if total is None else total + part
    assert rel_l2(total.cpu().numpy(), case["out"]) < TOL


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_reduced_precision_storage_matches_oracle_on_rounded_inputs(dtype):
    """Network outputs stored in bf16/fp16 are upcast exactly in-kernel, so the
    render matches the oracle fed the same rounded values."""
    case = Case("c3_s0")
    inp = case.inputs()
    w = case.workload
    attn_r = torch.from_numpy(inp["attn"]).to(dtype)
    sig_r = torch.from_numpy(inp["signal"]).to(dtype)
    torch.manual_seed(case.seed)
    ref = orc.render_spectrum(orc.RenderConfig.from_kwargs(**w.render),
                              orc.StubNetwork(attn_r.float(), sig_r.float()),
                              torch.from_numpy(inp["rays_o"]), torch.from_numpy(inp["position_tx"]),
                              torch.from_numpy(inp["direction_tx"])).numpy()
    a = attn_r.to(DEV).requires_grad_(True)
    sgn = sig_r.to(DEV).requires_grad_(True)
    r = AVRRender(Net(a, sgn), **w.render)
    torch.manual_seed(case.seed)
    out = r(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV),
            torch.from_numpy(inp["direction_tx"]).to(DEV))
    assert rel_l2(out.detach().cpu().numpy(), ref) < TOL
    (out * torch.from_numpy(case.grad_probe()).to(DEV)).sum().backward()
    assert sgn.grad.dtype == dtype and a.grad.dtype == dtype
    # gradients agree with the fp32 path up to the storage rounding
    a32 = torch.from_numpy(inp["attn"]).to(DEV).requires_grad_(True)
    s32 = torch.from_numpy(inp["signal"]).to(DEV).requires_grad_(True)
    r32 = AVRRender(Net(a32, s32), **w.render)
    torch.manual_seed(case.seed)
    o32 = r32(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV),
              torch.from_numpy(inp["direction_tx"]).to(DEV))
    (o32 * torch.from_numpy(case.grad_probe()).to(DEV)).sum().backward()
    gs, gs32 = sgn.grad.float().cpu().numpy(), s32.grad.cpu().numpy()
    tol = 2e-2 if dtype == torch.bfloat16 else 3e-3
    assert rel_l2(gs, gs32) < tol


def _nan_render(inp, w, seed, edit=None, **kw):
    sig = torch.from_numpy(inp["signal"]).to(DEV).clone()
    attn = torch.from_numpy(inp["attn"]).to(DEV).clone()
    if edit is not None:
        edit(attn, sig)
    r = AVRRender(Net(attn, sig), **w.render, **kw)
    torch.manual_seed(seed)
    with torch.no_grad():
        return r(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV))


def test_nonfinite_semantics():
    """Masked-region NaN/Inf (whole 16-byte chunks outside [delay, T-1-shift))
    is never loaded: the spectrum is exactly the clean one (the reference
    would give NaN, renderer.py:82,89).  A NaN in the live window gives NaN as
    in the reference.  propagate_nonfinite=True reproduces the reference in
    both cases ('Non-finite network outputs')."""
    case = Case("c1_s1")
    w, inp = case.workload, case.inputs()
    R, S, T = w.n_rays, w.n_samples, w.T
    delay, shift = case["delay"][0].astype(int), case["shift"].astype(int)
    assert delay.min() >= 4 and (shift >= 4).any()
    s_tail = int(np.nonzero(shift >= 4)[0][0])
    live = [(r, s) for r in range(R) for s in range(S) if delay[r, s] < T - 1 - shift[s]]
    assert live
    r_live, s_live = live[len(live) // 2]

    def masked(attn, sig):
        sig[0, 5 * S + 7, 0] = float("nan")          # t=0 < delay: a fully masked chunk
        sig[0, 9 * S + s_tail, T - 1] = float("inf")  # t >= T-1-shift: fully masked tail chunk

    def live_nan(attn, sig):
        sig[0, r_live * S + s_live, delay[r_live, s_live]] = float("nan")

    clean = _nan_render(inp, w, case.seed)
    assert torch.isfinite(clean).all()
    assert torch.equal(_nan_render(inp, w, case.seed, masked), clean)
    assert torch.isnan(_nan_render(inp, w, case.seed, live_nan)).any()
    strict = _nan_render(inp, w, case.seed, masked, propagate_nonfinite=True)
    assert torch.isnan(strict).all()
    assert torch.equal(_nan_render(inp, w, case.seed, None, propagate_nonfinite=True), clean)


@pytest.mark.parametrize("F", [2, 3, 128, 512, 801, 2048])
def test_spectrum_to_ir_gradient_matches_torch_irfft(F):
    """spectrum_to_ir's backward (avr_irfft_bwd) equals torch.fft.irfft's
    autograd (utils/criterion.py:71-72: the loss is taken on the IR), DC and
    Nyquist imaginary parts included (their gradient is zero)."""
    from avr_amd import spectrum_to_ir

    g = torch.Generator(device=DEV).manual_seed(F)
    B = 3
    spec = torch.randn(B, F, 2, device=DEV, generator=g)
    probe = torch.randn(B, 2 * (F - 1), device=DEV, generator=g)
    a = spec.clone().requires_grad_(True)
    ir = spectrum_to_ir(a)
    (ir * probe).sum().backward()
    b = spec.double().clone().requires_grad_(True)
    ir_ref = torch.real(torch.fft.irfft(b[..., 0] + 1j * b[..., 1], dim=-1))
    (ir_ref * probe.double()).sum().backward()
    assert ir.shape == ir_ref.shape
    assert rel_l2(ir.detach().double().cpu(), ir_ref.detach().cpu()) < 1e-5
    assert rel_l2(a.grad.double().cpu(), b.grad.cpu()) < 1e-5, rel_l2(a.grad.double().cpu(), b.grad.cpu())
    assert torch.all(a.grad[:, 0, 1] == 0) and torch.all(a.grad[:, -1, 1] == 0)


def test_render_ir_differentiable():
    """render_ir with autograd recording returns an IR that carries the
    gradient to the network outputs (the same as differentiating the
    spectrum through torch's irfft)."""
    case = Case("c1_s1")
    w, inp = case.workload, case.inputs()
    attn = torch.from_numpy(inp["attn"]).to(DEV).requires_grad_(True)
    sig = torch.from_numpy(inp["signal"]).to(DEV).requires_grad_(True)
    r = AVRRender(Net(attn, sig), **w.render)
    torch.manual_seed(case.seed)
    out, ir = r.render_ir(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV))
    probe = torch.linspace(-1, 1, ir.numel(), device=DEV).view_as(ir)
    (ir * probe).sum().backward()
    gs, ga = sig.grad.clone(), attn.grad.clone()
    sig.grad = attn.grad = None
    torch.manual_seed(case.seed)
    out2 = r(torch.from_numpy(inp["rays_o"]).to(DEV), torch.from_numpy(inp["position_tx"]).to(DEV))
    ir2 = torch.fft.irfft(out2[..., 0] + 1j * out2[..., 1], dim=-1)
    (ir2 * probe).sum().backward()
    assert rel_l2(gs.cpu(), sig.grad.cpu()) < 1e-4 and rel_l2(ga.cpu(), attn.grad.cpu()) < 1e-4
