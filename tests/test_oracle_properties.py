"""CPU property tests (hypothesis) of the render oracle over random small
configurations: the structural facts the HIP kernels are built on
 hold for the reference's algorithm at any shape, not only at
the golden ones.

* The spectrum is linear in the network's signal, so the reduction may be
  reordered (rays summed before the DFT, feature blocks summed in the fused
  head, ray shards all-reduced).
* Signal entries outside a row's live window [delay, T-1-shift) never reach
  the output, so the kernels do not read them.
* The compositing weights are non-negative and sum to at most 1 per ray
  (plus the reference's 1e-6 per transmittance factor).
"""
import numpy as np
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import avr_oracle as orc

from avr_amd.workloads import MESHRIR, RAF, SIMU


@st.composite
def render_cases(draw):
    """(cfg, T, B, seed): render blocks of the reference YAMLs with random
    ray / sample counts, a shorter `far`, and an even T long enough for the
    path-loss rows (shift <= 1.5 T, renderer.py:96-100)."""
    base = dict(draw(st.sampled_from([MESHRIR, RAF, SIMU])))
    base["far"] = draw(st.floats(0.25, float(base["far"])))
    base.update(n_azi=draw(st.integers(1, 6)), n_ele=draw(st.integers(1, 4)),
                n_samples=draw(st.integers(2, 24)))
    shift_max = int(round(base["fs"] * base["far"] / base["speed"]))
    t_min = max(16, -(-2 * shift_max // 3) + 4)
    T = 2 * draw(st.integers(t_min // 2 + 1, t_min // 2 + 48))
    return orc.RenderConfig.from_kwargs(**base), T, draw(st.integers(1, 2)), draw(st.integers(0, 2 ** 16))


def inputs(cfg, T, B, seed):
    rng = np.random.default_rng(seed)
    RS = cfg.n_rays * cfg.n_samples
    ro = torch.from_numpy(rng.uniform(-2, 2, (B, 3)).astype(np.float32))
    tx = torch.from_numpy(rng.uniform(-2, 2, (B, 3)).astype(np.float32))
    attn = torch.from_numpy(rng.uniform(0, 2, (B, RS, 1)).astype(np.float32))
    sig = torch.from_numpy((rng.standard_normal((B, RS, T)) * 0.1).astype(np.float32))
    return ro, tx, attn, sig


def render(cfg, attn, sig, ro, tx, seed, record=None):
    torch.manual_seed(seed)  # the azimuth jitter draw
    return orc.render_spectrum(cfg, orc.StubNetwork(attn, sig), ro, tx, record=record)


SETTINGS = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@SETTINGS
@given(render_cases())
def test_spectrum_is_linear_in_signal(case):
    cfg, T, B, seed = case
    ro, tx, attn, x1 = inputs(cfg, T, B, seed)
    x2 = torch.roll(x1, 1, dims=-1) * 0.7
    a = render(cfg, attn, x1, ro, tx, seed)
    b = render(cfg, attn, x2, ro, tx, seed)
    ab = render(cfg, attn, x1 + 2.5 * x2, ro, tx, seed)
    ref = a + 2.5 * b
    scale = float(a.norm() + 2.5 * b.norm()) + 1e-30
    assert float((ab - ref).norm()) <= 1e-5 * scale


@SETTINGS
@given(render_cases())
def test_entries_outside_the_live_window_do_not_matter(case):
    cfg, T, B, seed = case
    ro, tx, attn, sig = inputs(cfg, T, B, seed)
    rec = {}
    out = render(cfg, attn, sig, ro, tx, seed, rec)
    R, S = cfg.n_rays, cfg.n_samples
    t = torch.arange(T)
    delay = rec["delay"].reshape(B, R, S, 1)
    lim = (T - 1 - rec["shift"]).reshape(1, 1, S, 1)
    live = (t >= delay) & (t < lim)
    noise = torch.randn(sig.shape, generator=torch.Generator().manual_seed(seed)) * 5
    other = torch.where(live.reshape(B, R * S, T), sig, noise)
    assert torch.equal(render(cfg, attn, other, ro, tx, seed), out)


@SETTINGS
@given(render_cases())
def test_weights_are_a_sub_partition_of_unity(case):
    cfg, T, B, seed = case
    ro, tx, attn, sig = inputs(cfg, T, B, seed)
    rec = {}
    render(cfg, attn, sig, ro, tx, seed, rec)
    w = rec["weights"]
    assert bool((w >= 0).all())
    assert float(w.sum(-1).max()) <= 1.0 + cfg.n_samples * 1e-6 + 1e-6
