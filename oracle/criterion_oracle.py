"""CPU oracle for the training criterion — TEST INFRASTRUCTURE ONLY.

Only `tests/` may import this module; the product criterion
(`avr_amd.criterion.Criterion`) runs HIP kernels and never calls it.

Op-for-op torch-CPU restatement of `utils/criterion.py:69-126` (the loss the
training loop applies to the rendered spectrum, avr_runner.py:181) including
the multi-resolution STFT loss it takes from the third-party package
`auraloss` (criterion.py:3, 33; requirements.txt:6, unpinned, so the current
release 0.4.0 is restated here):

  auraloss.freq.MultiResolutionSTFTLoss(fft_sizes, hop_sizes, win_lengths,
      window="hann_window", w_sc=1, w_log_mag=1, w_lin_mag=<given>, w_phs=0,
      eps=1e-8, reduction="mean", mag_distance="L1")
    forward(x, y) = mean over resolutions of STFTLoss_i(x, y)
  STFTLoss.forward(x, y):
    X = torch.stft(x, n_fft, hop, win_length, hann_window(win_length),
                   return_complex=True)          (center, reflect padding)
    mag = sqrt(clamp(re^2 + im^2, min=eps))
    sc  = mean_b ||mag_y - mag_x||_F / ||mag_y||_F   (norm over the last 2 dims)
    log = L1(log(mag_x), log(mag_y)),  lin = L1(mag_x, mag_y)
    loss = w_sc*sc + w_log_mag*log + w_lin_mag*lin

Parity status: criterion.py cannot be imported here (auraloss and librosa
are absent; an ordinary ImportError), so this restatement is NOT pinned to
the running reference: "parity unpinned".  The spectral / time / energy terms
are written with the exact torch ops of criterion.py:71-96; the MR-STFT term
follows auraloss 0.4.0's published algorithm as summarised above.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# criterion.py:33
MR_FFT_SIZES = (512, 256, 128, 64)
MR_WIN_LENGTHS = (300, 150, 75, 30)
MR_HOP_SIZES = (60, 30, 8, 4)
MR_EPS = 1e-8
# criterion.py:74 (torch.stft defaults: hop n_fft//4, rectangular window)
ENERGY_NFFT = 256

LOSS_KEYS = ("spec_loss_weight", "amplitude_loss_weight", "angle_loss_weight",
             "time_loss_weight", "energy_loss_weight", "multistft_loss_weight")


def _stft_mag(x, n_fft, hop, win_length, eps):
    """auraloss STFTLoss.stft: magnitude sqrt(clamp(|X|^2, eps))."""
    window = torch.hann_window(win_length).to(x.device)
    X = torch.stft(x, n_fft, hop, win_length, window, return_complex=True)
    return torch.sqrt(torch.clamp((X.real ** 2) + (X.imag ** 2), min=eps))


def stft_loss(x, y, n_fft, hop, win_length, w_sc=1.0, w_log=1.0, w_lin=1.0, eps=MR_EPS):
    """auraloss.freq.STFTLoss(...)(x, y) for x, y [B, 1, T]."""
    x_mag = _stft_mag(x.view(-1, x.size(-1)), n_fft, hop, win_length, eps)
    y_mag = _stft_mag(y.view(-1, y.size(-1)), n_fft, hop, win_length, eps)
    sc = (torch.norm(y_mag - x_mag, p="fro", dim=[-1, -2]) /
          torch.norm(y_mag, p="fro", dim=[-1, -2])).mean()
    log = F.l1_loss(torch.log(x_mag), torch.log(y_mag))
    lin = F.l1_loss(x_mag, y_mag)
    return w_sc * sc + w_log * log + w_lin * lin


def mr_stft_loss(x, y):
    """auraloss.freq.MultiResolutionSTFTLoss(w_lin_mag=1, criterion.py:33)."""
    total = 0.0
    for n_fft, win, hop in zip(MR_FFT_SIZES, MR_WIN_LENGTHS, MR_HOP_SIZES):
        total = total + stft_loss(x, y, n_fft, hop, win)
    return total / len(MR_FFT_SIZES)


def energy_decay(time_sig):
    """criterion.py:74-83: log10 energy decay curve of |STFT|^2 frame energy."""
    spec = torch.abs(torch.stft(time_sig, n_fft=ENERGY_NFFT, return_complex=True))
    e = torch.sum(spec ** 2, dim=1)
    curve = torch.log10(torch.flip(torch.cumsum(torch.flip(e, [-1]) ** 2, dim=-1), [-1]) + 1e-9)
    curve = curve - curve[:, [0]]
    return curve


def criterion(pred_sig, ori_sig, weights):
    """utils/criterion.py:69-126 without the DAS branch (weights 0 by default).

    pred_sig, ori_sig: complex [B, F].  weights: dict with LOSS_KEYS.
    Returns (spec, amplitude, angle, time, energy, multi_stft, ori_time, pred_time).
    """
    l1 = F.l1_loss
    pred_time = torch.real(torch.fft.irfft(pred_sig, dim=-1))
    ori_time = torch.real(torch.fft.irfft(ori_sig, dim=-1))
    predict_energy = energy_decay(pred_time)
    ori_energy = energy_decay(ori_time)

    real_loss = l1(torch.real(pred_sig), torch.real(ori_sig))
    imag_loss = l1(torch.imag(pred_sig), torch.imag(ori_sig))
    spec = (real_loss + imag_loss) * weights["spec_loss_weight"]
    amp = l1(torch.abs(pred_sig), torch.abs(ori_sig)) * weights["amplitude_loss_weight"]
    angle = (l1(torch.cos(torch.angle(pred_sig)), torch.cos(torch.angle(ori_sig))) +
             l1(torch.sin(torch.angle(pred_sig)), torch.sin(torch.angle(ori_sig)))) \
        * weights["angle_loss_weight"]
    time = l1(ori_time, pred_time) * weights["time_loss_weight"]
    energy = l1(ori_energy, predict_energy) * weights["energy_loss_weight"]
    mr = mr_stft_loss(ori_time.unsqueeze(1), pred_time.unsqueeze(1)) * weights["multistft_loss_weight"]
    return spec, amp, angle, time, energy, mr, ori_time, pred_time


def beamforming_power(sig, fs, speed, n_fft=512):
    """Criterion.compute_beamforming_power (criterion.py:35-67): DAS power over
    360 one-degree look directions for an 8-microphone circular array."""
    M = sig.shape[0]
    assert M == 8, f"Expected 8 microphones, but got {M}"
    angles_rad = torch.deg2rad(torch.arange(0.0, 360.0, 1.0))
    time_sig = torch.real(torch.fft.irfft(sig, dim=-1))
    freqs = torch.fft.rfftfreq(n_fft, 1 / fs)
    X = torch.fft.rfft(time_sig, n=n_fft, dim=-1)
    mic_angles = torch.linspace(math.pi / 2, math.pi / 2 + 2 * math.pi, M + 1)[:-1]
    mic_pos = torch.stack([torch.cos(mic_angles), torch.sin(mic_angles)], dim=-1)
    mic_pos -= mic_pos.mean(dim=0)
    steering = torch.zeros(len(angles_rad), M, X.shape[1], dtype=torch.cfloat)
    for i, theta in enumerate(angles_rad):
        u = torch.tensor([torch.cos(theta), torch.sin(theta)])
        delays = (mic_pos @ u) / speed
        steering[i] = torch.exp(-1j * 2 * math.pi * delays[:, None] * freqs[None, :])
    beam = torch.einsum('mf,kmf->kf', X, steering) / M
    beam_power = torch.abs(beam) ** 2
    beam_power_norm = beam_power / (torch.sum(beam_power, dim=0, keepdim=True) + 1e-8)
    return torch.sum(beam_power_norm, dim=-1)


def das_losses(pred_sig, ori_sig, fs, speed, reg_weight, ce_weight, beta=100.0):
    """criterion.py:100-122: DAS regression / cross-entropy terms."""
    angles_rad = torch.deg2rad(torch.arange(0.0, 360.0, 1.0))
    reg = torch.tensor(0.0)
    ce = torch.tensor(0.0)
    if reg_weight > 0 or ce_weight > 0:
        pp = beamforming_power(pred_sig, fs, speed)
        po = beamforming_power(ori_sig, fs, speed)
        if ce_weight > 0:
            target = torch.argmax(po).unsqueeze(0)
            ce = F.cross_entropy(pp.unsqueeze(0), target) * ce_weight
        if reg_weight > 0:
            wp = torch.softmax(beta * pp, dim=0)
            wo = torch.softmax(beta * po, dim=0)
            a_p = torch.sum(wp * angles_rad)
            a_o = torch.sum(wo * angles_rad)
            reg = (F.l1_loss(torch.sin(a_p), torch.sin(a_o)) +
                   F.l1_loss(torch.cos(a_p), torch.cos(a_o))) * reg_weight
    return reg, ce
