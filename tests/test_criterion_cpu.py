"""CPU: the criterion oracle (oracle/criterion_oracle.py) checked against an
independent numpy statement of the same transforms, and the product
criterion's host-side contract (no compute without a GPU).

Every term except the MR-STFT one (and the gradient of their sum) is
pinned to golden vectors of the reference's own utils/criterion.py
(tests/golden/criterion, tools/gen_criterion_golden.py).  The MR-STFT term
cannot be (auraloss is absent here): for it these tests pin the
restatement's reading of torch.stft's conventions (centre reflect padding, a
short window centred in n_fft, hop defaults, one-sided bins) and of the loss
formulas."""
import numpy as np
import pytest
import torch

from oracle import criterion_oracle as co

pytestmark = pytest.mark.filterwarnings("ignore::UserWarning")


def _np_stft(x, n_fft, hop, window):
    """Direct DFT of reflect-padded frames with a centred window (float64)."""
    pad = n_fft // 2
    xp = np.pad(x, (pad, pad), mode="reflect")
    w = np.zeros(n_fft)
    off = (n_fft - len(window)) // 2
    w[off:off + len(window)] = window
    M = 1 + len(x) // hop
    k = np.arange(n_fft // 2 + 1)[:, None]
    t = np.arange(n_fft)[None, :]
    basis = np.exp(-2j * np.pi * k * t / n_fft)
    return np.stack([basis @ (w * xp[m * hop:m * hop + n_fft]) for m in range(M)], axis=1)


def _np_hann(L):
    return 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(L) / L)  # periodic


def _signals(B=2, n=600, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = rng.standard_normal((B, n)) * np.exp(-t / 150.0)
    y = x + 0.3 * rng.standard_normal((B, n)) * np.exp(-t / 150.0)
    return x, y


def test_stft_conventions_match_numpy():
    x, _ = _signals(1, 600)
    for n_fft, win, hop in zip(co.MR_FFT_SIZES, co.MR_WIN_LENGTHS, co.MR_HOP_SIZES):
        ref = _np_stft(x[0], n_fft, hop, _np_hann(win))
        X = torch.stft(torch.from_numpy(x).double(), n_fft, hop, win,
                       torch.hann_window(win, dtype=torch.float64), return_complex=True)[0]
        assert X.shape == ref.shape
        assert np.abs(X.numpy() - ref).max() < 1e-9 * np.abs(ref).max()


def test_mr_stft_loss_matches_numpy():
    x, y = _signals(2, 700, 1)
    total = 0.0
    for n_fft, win, hop in zip(co.MR_FFT_SIZES, co.MR_WIN_LENGTHS, co.MR_HOP_SIZES):
        xm = np.stack([np.sqrt(np.maximum(np.abs(_np_stft(r, n_fft, hop, _np_hann(win))) ** 2, 1e-8))
                       for r in x])
        ym = np.stack([np.sqrt(np.maximum(np.abs(_np_stft(r, n_fft, hop, _np_hann(win))) ** 2, 1e-8))
                       for r in y])
        sc = np.mean([np.linalg.norm(ym[b] - xm[b]) / np.linalg.norm(ym[b]) for b in range(2)])
        lg = np.mean(np.abs(np.log(xm) - np.log(ym)))
        ln = np.mean(np.abs(xm - ym))
        total += sc + lg + ln
    total /= 4
    got = co.mr_stft_loss(torch.from_numpy(x).double().unsqueeze(1),
                          torch.from_numpy(y).double().unsqueeze(1))
    assert abs(float(got) - total) < 1e-6 * total  # auraloss builds an fp32 hann window


def test_energy_decay_matches_numpy():
    x, _ = _signals(2, 800, 2)
    e = np.stack([np.sum(np.abs(_np_stft(r, 256, 64, np.ones(256))) ** 2, axis=0) for r in x])
    c = np.cumsum((e ** 2)[:, ::-1], axis=1)[:, ::-1]
    curve = np.log10(c + 1e-9)
    curve = curve - curve[:, :1]
    got = co.energy_decay(torch.from_numpy(x).double())
    assert np.abs(got.numpy() - curve).max() < 1e-9


def test_criterion_terms_match_formulas():
    """Spectral / time terms against their definitions (criterion.py:85-94)."""
    rng = np.random.default_rng(3)
    B, F = 2, 257
    p = rng.standard_normal((B, F)) + 1j * rng.standard_normal((B, F))
    o = rng.standard_normal((B, F)) + 1j * rng.standard_normal((B, F))
    w = dict(zip(co.LOSS_KEYS, [1.0, 0.5, 0.25, 10.0, 0.0, 0.0]))
    out = co.criterion(torch.from_numpy(p), torch.from_numpy(o), w)
    spec = np.mean(np.abs(p.real - o.real)) + np.mean(np.abs(p.imag - o.imag))
    amp = 0.5 * np.mean(np.abs(np.abs(p) - np.abs(o)))
    ang = 0.25 * (np.mean(np.abs(np.cos(np.angle(p)) - np.cos(np.angle(o)))) +
                  np.mean(np.abs(np.sin(np.angle(p)) - np.sin(np.angle(o)))))
    tm = 10.0 * np.mean(np.abs(np.fft.irfft(o) - np.fft.irfft(p)))
    for got, want in zip(out[:4], (spec, amp, ang, tm)):
        assert abs(float(got) - want) < 1e-9 * max(1.0, abs(want))


def test_das_power_is_a_distribution_over_directions_per_bin():
    """sum_k bpn[k, f] = 1 for every bin with energy, so sum_k power = #bins."""
    rng = np.random.default_rng(4)
    sig = torch.from_numpy(rng.standard_normal((8, 257)) + 1j * rng.standard_normal((8, 257)))
    power = co.beamforming_power(sig.to(torch.complex64), 16000, 343.0)
    assert power.shape == (360,)
    assert abs(float(power.sum()) - 257) < 1e-2


def test_product_criterion_refuses_cpu_tensors():
    from avr_amd.criterion import Criterion
    w = dict(zip(co.LOSS_KEYS, [1, 1, 1, 1, 1, 1]))
    crit = Criterion(w, dict(fs=16000, speed=343.0))
    x = torch.zeros(1, 257, dtype=torch.complex64)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        crit(x, x)


@pytest.mark.parametrize("name", [c[0] for c in __import__("criterion_cases").CASES])
def test_oracle_matches_reference_criterion_golden(name):
    """The restatement against golden vectors of the reference's own
    utils/criterion.py (tools/gen_criterion_golden.py): every term except the
    auraloss MR-STFT one, and the gradient of their sum."""
    import os

    from criterion_cases import CASES, RENDER, spectra

    case = {c[0]: c for c in CASES}[name]
    _, B, F, weights, seed = case
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "criterion",
                             f"crit_{name}.npz"))
    pred, ori = spectra(B, F, seed)
    p = pred.clone().requires_grad_(True)
    o = co.criterion(p, ori, weights)
    terms = list(o[:5]) + list(co.das_losses(p, ori, RENDER["fs"], RENDER["speed"],
                                             weights.get("das_reg_loss_weight", 0.0),
                                             weights.get("das_ce_loss_weight", 0.0),
                                             weights.get("beta", 100.0)))
    np.testing.assert_allclose([float(x) for x in terms], z["losses"], rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(o[6].numpy(), z["ori_time"])
    np.testing.assert_array_equal(o[7].detach().numpy(), z["pred_time"])
    sum(terms).backward()
    np.testing.assert_allclose(torch.view_as_real(p.grad).numpy(), z["grad"], rtol=1e-5, atol=1e-9)
