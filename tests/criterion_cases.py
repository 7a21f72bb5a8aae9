"""Criterion test cases shared by the GPU tests and
tools/gen_criterion_golden.py (which writes tests/golden/criterion/ from the
reference's utils/criterion.py): seeded spectra and the loss weights of the
reference configs."""
import numpy as np
import torch

MESHRIR_W = dict(spec_loss_weight=1, amplitude_loss_weight=0.5, angle_loss_weight=0.5,
                 time_loss_weight=100, energy_loss_weight=5, multistft_loss_weight=1)
RAF_W = dict(spec_loss_weight=1, amplitude_loss_weight=1, angle_loss_weight=1,
             time_loss_weight=20, energy_loss_weight=3, multistft_loss_weight=2)
# config_files/avr_real_exp_ch_emb_add_das_optuna.yml: DAS regression on, CE off
DAS_REG_W = dict(RAF_W, das_reg_loss_weight=1, das_ce_loss_weight=0, beta=100)
DAS_BOTH_W = dict(RAF_W, das_reg_loss_weight=0.5, das_ce_loss_weight=0.25, beta=100)
RENDER = dict(fs=16000, speed=346.8)

CASES = [
    # name, B, F, weights, seed
    ("meshrir_c2", 2, 512, MESHRIR_W, 0),
    ("raf_c3", 4, 801, RAF_W, 1),
    ("raf_c4", 4, 801, MESHRIR_W, 2),
    ("simu_long", 1, 2048, RAF_W, 3),
    ("min_len", 3, 130, RAF_W, 4),  # n = 258: smallest IR the 512-point STFT accepts
    ("das_reg", 8, 801, DAS_REG_W, 5),  # 8 microphones (criterion.py:41)
    ("das_both", 8, 401, DAS_BOTH_W, 6),
]


def spectra(B, F, seed, noise=0.3):
    """A decaying-noise IR's spectrum (ori) and a perturbed copy (pred)."""
    rng = np.random.default_rng(seed)
    n = 2 * (F - 1)
    t = np.arange(n)
    ir = rng.standard_normal((B, n)) * np.exp(-t / (0.15 * n)) * 0.05
    ori = torch.fft.rfft(torch.from_numpy(ir).float())
    pert = torch.from_numpy(rng.standard_normal((B, F)) + 1j * rng.standard_normal((B, F)))
    pred = ori + noise * ori.abs().mean() * pert.to(torch.complex64)
    return pred.to(torch.complex64), ori.to(torch.complex64)
