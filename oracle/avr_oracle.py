"""CPU oracle for the AVR render hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the HIP product path.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it;
the product package `avr_amd` never does (it fails loudly without its HIP
library instead of falling back here).

It is an op-for-op torch-CPU restatement of the reference renderer
(`/root/reference/renderer_cpu.py`, identical math to `renderer.py`), written
stage by stage so each step can be checked on its own.  Every torch op is the
one the reference issues, in the same order and dtype, so results are
bit-identical to the reference on the same inputs (pinned by
`tests/golden/*.npz`, produced by `tools/gen_golden.py`, which imports the
real reference in the build container).

Parity status: PINNED against golden vectors generated from the reference
itself (see tests/test_oracle_golden.py).  The hash-grid encoding is NOT part
of this file (tinycudann is absent: see oracle/hashgrid_oracle.py, "parity
unpinned").
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

__all__ = [
    "RenderConfig",
    "sphere_directions",
    "depth_samples",
    "to_unit_cube",
    "from_unit_cube",
    "receiver_delay",
    "tail_keep_mask",
    "source_delay",
    "path_loss_table",
    "path_loss_rows",
    "phase_rotation",
    "composite_weights",
    "network_inputs",
    "render_spectrum",
    "spectrum_to_ir",
]


@dataclass
class RenderConfig:
    """The `render:` keys AVRRender reads (renderer_cpu.py:11-21)."""

    n_samples: int
    near: float
    far: float
    n_azi: int
    n_ele: int
    speed: float
    fs: float
    pathloss: float
    xyz_min: float
    xyz_max: float

    @classmethod
    def from_kwargs(cls, **kw):
        return cls(**{k: kw[k] for k in cls.__dataclass_fields__})

    @property
    def n_rays(self) -> int:
        return self.n_azi * self.n_ele + 2


# --------------------------------------------------------------------------
# a2: spherical ray directions  (renderer_cpu.py:111-143, renderer.py:133-165)
# --------------------------------------------------------------------------
def sphere_directions(n_azi: int, n_ele: int, jitter=True):
    """Ray directions [n_azi*n_ele+2, 3] plus the azimuth jitter draw.

    The jitter consumes `torch.rand(n_azi)` and then `torch.rand(n_ele)` from
    the CPU default generator (renderer_cpu.py:127,131; on the GPU path too,
    renderer.py:149,153).  The elevation draw is multiplied by zero but still
    advances the generator.  Returns (dirs, u_azi) with u_azi the raw U[0,1)
    draw so the HIP path can be fed the identical values.
    """
    two_pi = np.pi * 2
    base_azi = torch.linspace(0, two_pi, n_azi + 1)[:-1]
    u_azi = torch.rand(n_azi)
    shift = (two_pi / n_azi) * u_azi
    azi = base_azi + shift if jitter else base_azi
    u_ele = torch.rand(n_ele)
    ele_lin = torch.linspace(0, 1, n_ele + 2)[1:-1] + (0.5 / n_ele) * u_ele * 0
    ele = torch.acos(2 * ele_lin - 1)
    grid_a, grid_e = torch.meshgrid(azi, ele, indexing="ij")
    ga, ge = grid_a.flatten(), grid_e.flatten()
    sin_e = torch.sin(ge)
    xyz = torch.cat(
        (
            torch.mul(torch.cos(ga), sin_e).unsqueeze(1),
            torch.mul(torch.sin(ga), sin_e).unsqueeze(1),
            torch.cos(ge).unsqueeze(1),
        ),
        dim=1,
    )
    poles = torch.tensor([[0, 0, 1], [0, 0, -1]])
    return torch.cat((xyz, poles), dim=0), u_azi


# --------------------------------------------------------------------------
# a3/a4: sampling and coordinate maps (renderer_cpu.py:46-54, 105-109)
# --------------------------------------------------------------------------
def depth_samples(cfg: RenderConfig):
    """d_vals [S] = linspace(0,1,S)*(far-near)+near (renderer_cpu.py:46)."""
    return torch.linspace(0.0, 1.0, cfg.n_samples) * (cfg.far - cfg.near) + cfg.near


def to_unit_cube(p, lo, hi):
    """normalize_points (renderer_cpu.py:105-106): 2*(p-lo)/(hi-lo)-1."""
    return 2 * (p - lo) / (hi - lo) - 1


def from_unit_cube(q, lo, hi):
    """denormalize_points (renderer_cpu.py:108-109): (q+1)/2*(hi-lo)+lo."""
    return (q + 1) / 2 * (hi - lo) + lo


def network_inputs(cfg: RenderConfig, rays_o, position_tx, dirs, d_vals, direction_tx=None):
    """Tensors handed to network_fn (renderer_cpu.py:47-54).

    Returns (pts, view, tx, dir_tx) each [B, R*S, 3] (dir_tx None if absent).
    """
    B = position_tx.size(0)
    along = (dirs.unsqueeze(1) * d_vals.unsqueeze(0).unsqueeze(2)).unsqueeze(0)
    world = rays_o.unsqueeze(1).unsqueeze(2) + along  # [B,R,S,3]
    pts = to_unit_cube(world.reshape(B, -1, 3), cfg.xyz_min, cfg.xyz_max)
    view = -1 * dirs.unsqueeze(0).unsqueeze(2).expand(world.size()).reshape(B, -1, 3)
    tx = to_unit_cube(position_tx.unsqueeze(1).expand(*pts.size()), cfg.xyz_min, cfg.xyz_max)
    dtx = None
    if direction_tx is not None:
        dtx = direction_tx.unsqueeze(1).expand(*pts.size())
    return pts, view, tx, dtx


# --------------------------------------------------------------------------
# a7/a8: integer delays and masks (renderer_cpu.py:69-80)
# --------------------------------------------------------------------------
def receiver_delay(cfg: RenderConfig, d_vals):
    """(pts2rx_idx [S] fp32, shift [S] fp32-rounded) — renderer_cpu.py:69-70."""
    frac = cfg.fs * d_vals / cfg.speed
    return frac, torch.round(frac)


def tail_keep_mask(shift, T: int):
    """int64 [S,T]: 1 where (T-1-t) - shift[s] > 0 (renderer_cpu.py:72)."""
    rev = torch.arange(T - 1, 0 - 1, -1).unsqueeze(0)
    return torch.where((rev - shift.unsqueeze(1)) > 0, 1, 0)


def source_delay(cfg: RenderConfig, tx_n, pts_n, B: int, S: int, T: int):
    """Integer tx->point delay per ray-sample, [B,R,S,1] fp32 (renderer_cpu.py:76-77).

    Computed from the *normalized* network inputs, exactly as the reference
    does (the denormalize round trip re-adds (lo+hi)/2).
    """
    world_gap = from_unit_cube(tx_n - pts_n, cfg.xyz_min, cfg.xyz_max)
    samples = torch.linalg.vector_norm(world_gap, dim=-1).reshape(B, -1, S) * cfg.fs / cfg.speed
    return torch.clamp(torch.round(samples), min=0, max=T - 1).unsqueeze(-1)


# --------------------------------------------------------------------------
# a9: 1/d path loss gathered at shift[s]+t (renderer_cpu.py:83-87)
# --------------------------------------------------------------------------
def path_loss_table(cfg: RenderConfig, T: int):
    """The 1/d table of ceil(2.5T) entries with the near-field clamp."""
    near_n = int(0.1 / cfg.speed * cfg.fs)
    dist = torch.arange(0, T * 2.5, device="cpu") / cfg.fs * cfg.speed
    table = cfg.pathloss / (dist + 1e-3)
    table[0:near_n] = table[near_n + 1]
    return table


def path_loss_rows(cfg: RenderConfig, shift, T: int):
    """[S,T] rows table[shift[s] : shift[s]+T]; raises like torch.stack when a
    row would run off the table (shift > 1.5T)."""
    table = path_loss_table(cfg, T)
    starts = shift.detach().cpu().numpy().astype(int)
    return torch.stack([table[i : i + T] for i in starts])


# --------------------------------------------------------------------------
# a10: fractional-delay phase (renderer_cpu.py:91)
# --------------------------------------------------------------------------
def phase_rotation(frac, T: int):
    """complex64 [S,F] = exp(-i*2*pi/T * f * pts2rx_idx[s])."""
    F = T // 2 + 1
    return torch.exp(-1j * 2 * np.pi / T * torch.arange(0, F).unsqueeze(0) * frac.unsqueeze(1))


# --------------------------------------------------------------------------
# a11: alpha compositing weights (renderer_cpu.py:145-171)
# --------------------------------------------------------------------------
def composite_weights(attn, d_vals):
    """w [B,R,S] = T_s * alpha_s with exclusive transmittance product."""
    B, R, S = attn.shape
    gaps = d_vals[..., 1:] - d_vals[..., :-1]
    gaps = torch.cat([gaps, torch.Tensor([1e10]).expand(gaps[..., :1].shape)], -1)
    gaps = gaps.unsqueeze(0).repeat(R, 1).repeat(B, 1, 1)
    alpha = 1.0 - torch.exp(-attn * gaps)
    factors = torch.cat([torch.ones(alpha[..., :1].shape), 1.0 - alpha + 1e-6], -1)
    trans = torch.cumprod(factors, -1)[..., :-1]
    return trans * alpha


# --------------------------------------------------------------------------
# Full forward (renderer_cpu.py:23-102) with a precomputed network output
# --------------------------------------------------------------------------
def render_spectrum(cfg: RenderConfig, network_fn, rays_o, position_tx, direction_tx=None,
                    record: dict | None = None):
    """Rendered spectrum [B, F, 2] fp32, the reference forward restated.

    `network_fn(pts, view, tx[, dir_tx]) -> (attn [B,R*S,1], signal [B,R*S,T])`.
    If `record` is a dict it receives the intermediates (dirs, u_azi, d_vals,
    frac, shift, delay, weights) for stage-level checks.
    """
    B = position_tx.size(0)
    S = cfg.n_samples
    dirs, u_azi = sphere_directions(cfg.n_azi, cfg.n_ele)
    d_vals = depth_samples(cfg)
    pts, view, tx, dtx = network_inputs(cfg, rays_o, position_tx, dirs, d_vals, direction_tx)
    if dtx is not None:
        attn, signal = network_fn(pts, view, tx, dtx)
    else:
        attn, signal = network_fn(pts, view, tx)
    attn = attn.to("cpu").view(B, -1, S)
    signal = signal.to("cpu")
    signal = signal.view(B, -1, S, signal.size(-1))
    T = signal.size(-1)

    frac, shift = receiver_delay(cfg, d_vals)
    signal = signal * tail_keep_mask(shift, T)
    delay = source_delay(cfg, tx, pts, B, S, T)
    signal = signal * (torch.arange(T) >= delay)

    rows = path_loss_rows(cfg, shift, T)
    spec = torch.fft.rfft(signal.float() * rows, dim=-1) * phase_rotation(frac, T)
    w = composite_weights(attn, d_vals)
    per_ray = torch.sum(spec * w[..., None], -2)
    total = torch.sum(per_ray, dim=-2)
    out = torch.cat([torch.real(total).unsqueeze(-1), torch.imag(total).unsqueeze(-1)], dim=-1)
    if record is not None:
        record.update(dirs=dirs, u_azi=u_azi, d_vals=d_vals, frac=frac, shift=shift,
                      delay=delay[..., 0], weights=w, pts=pts, view=view, tx=tx, dir_tx=dtx)
    return out


def spectrum_to_ir(out):
    """IR [B, T] from a [B, F, 2] spectrum: the caller's complex view
    (avr_runner.py:178) followed by Criterion's irfft (utils/criterion.py:71)."""
    z = out[..., 0] + 1j * out[..., 1]
    return torch.real(torch.fft.irfft(z, dim=-1))


class StubNetwork(torch.nn.Module):
    """network_fn stand-in returning fixed (attn, signal); records its inputs."""

    def __init__(self, attn, signal):
        super().__init__()
        self.attn, self.signal = attn, signal
        self.seen = None

    def forward(self, pts, view, tx, dir_tx=None, ch_idx=None):
        self.seen = (pts, view, tx, dir_tx)
        return self.attn, self.signal
