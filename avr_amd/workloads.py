"""Canonical render configurations and seeded synthetic inputs.

The five workloads of BASELINE.json `configs`, with the
`render:` blocks of the reference YAML files they are quoted on:

* MeshRIR (config_files/avr_meshrir.yml:11-21): xyz +-6, far 4, fs 24000,
  speed 343.8, pathloss 1.5
* RAF (config_files/avr_raf_furnished.yml:11-22): xyz +-12, far 6, fs 16000,
  speed 346.8, pathloss 0.5, speaker orientation present
* Simu (config_files/avr_simu.yml:11-21): xyz +-10, far 6, fs 16000,
  speed 343.8, pathloss 1.5

Inputs follow SURVEY.md §8(d): rays_o, position_tx ~ U(-2,2)^3,
direction_tx = normalised N(0,I), attn ~ U[0,2), signal ~ 0.1 N(0,1), all
drawn in that order from `np.random.default_rng(seed)` as float32.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field

import numpy as np

MESHRIR = dict(xyz_min=-6, xyz_max=6, near=0, far=4, speed=343.8, fs=24000, pathloss=1.5)
RAF = dict(xyz_min=-12, xyz_max=12, near=0, far=6, speed=346.8, fs=16000, pathloss=0.5)
SIMU = dict(xyz_min=-10, xyz_max=10, near=0, far=6, speed=343.8, fs=16000, pathloss=1.5)


@dataclass
class Workload:
    name: str
    render: dict
    T: int  # signal_output_dim
    batch: int
    with_dir_tx: bool = False
    signal_dtype: str = "float32"
    attn_dtype: str = "float32"
    note: str = ""

    @property
    def n_rays(self) -> int:
        return self.render["n_azi"] * self.render["n_ele"] + 2

    @property
    def n_samples(self) -> int:
        return self.render["n_samples"]

    @property
    def F(self) -> int:
        return self.T // 2 + 1

    @property
    def ray_samples(self) -> int:
        return self.batch * self.n_rays * self.n_samples

    def replace(self, **kw) -> "Workload":
        render = dict(self.render)
        for k in list(kw):
            if k in render:
                render[k] = kw.pop(k)
        return dataclasses.replace(self, render=render, **kw)


def _rcfg(base, n_azi, n_ele, n_samples, **over):
    r = dict(base)
    r.update(n_azi=n_azi, n_ele=n_ele, n_samples=n_samples)
    r.update(over)
    return r


WORKLOADS = {
    # configs[0]: plumbing case, CPU-runnable
    "c1_meshrir_plumbing": Workload("c1_meshrir_plumbing", _rcfg(MESHRIR, 6, 5, 64), 254, 1),
    # configs[1]: the headline metric's workload
    "c2_meshrir_1024x256x512": Workload("c2_meshrir_1024x256x512", _rcfg(MESHRIR, 73, 14, 256), 1022, 1),
    # configs[2]: RAF-Furnished training step, batch 4
    "c3_raf_furnished_b4": Workload("c3_raf_furnished_b4", _rcfg(RAF, 36, 18, 32), 1600, 4, with_dir_tx=True),
    # configs[3]: RAF-Empty, batch 32 over 8 GPUs = 4 per GPU (per-rank shard)
    "c4_raf_empty_b4_per_gpu": Workload("c4_raf_empty_b4_per_gpu", _rcfg(RAF, 48, 24, 32), 1600, 4, with_dir_tx=True),
    # configs[4]: long IR, fp16 network output storage
    "c5_simu_4096x512x2048": Workload("c5_simu_4096x512x2048", _rcfg(SIMU, 89, 46, 512), 4094, 1,
                                      signal_dtype="float16", attn_dtype="float16"),
}


def make_inputs(w: Workload, seed: int):
    """Seeded numpy inputs for workload `w` (draw order fixed, see module doc)."""
    rng = np.random.default_rng(seed)
    B, RS, T = w.batch, w.n_rays * w.n_samples, w.T
    rays_o = rng.uniform(-2.0, 2.0, size=(B, 3)).astype(np.float32)
    position_tx = rng.uniform(-2.0, 2.0, size=(B, 3)).astype(np.float32)
    direction_tx = None
    if w.with_dir_tx:
        v = rng.standard_normal(size=(B, 3)).astype(np.float32)
        direction_tx = (v / np.linalg.norm(v, axis=-1, keepdims=True)).astype(np.float32)
    attn = rng.uniform(0.0, 2.0, size=(B, RS, 1)).astype(np.float32)
    signal = rng.standard_normal(size=(B, RS, T), dtype=np.float32)
    signal *= np.float32(0.1)
    attn = attn.astype(w.attn_dtype)
    signal = signal.astype(w.signal_dtype, copy=False)
    return dict(rays_o=rays_o, position_tx=position_tx, direction_tx=direction_tx,
                attn=attn, signal=signal)


def grad_probe(w: Workload, seed: int):
    """Fixed upstream gradient dL/d(out) [B,F,2] used by the backward fixtures."""
    rng = np.random.default_rng(10_000 + seed)
    return rng.standard_normal(size=(w.batch, w.F, 2)).astype(np.float32)


def _grid(log2):
    return dict(otype="HashGrid", n_levels=20, n_features_per_level=2, log2_hashmap_size=log2,
                base_resolution=16)


def _mlp(n_hidden, width):
    return dict(otype="FullyFusedMLP", activation="ReLU", output_activation="None",
                n_neurons=width, n_hidden_layers=n_hidden)


# `model:` blocks of the reference configs (shapes only; weights are random)
MESHRIR_MODEL = dict(  # config_files/avr_meshrir.yml:44-89
    signal_output_dim=2400, leaky_relu=0.03,
    pos_encoding_sigma=_grid(18), dir_encoding_sig=_grid(20), tx_encoding_sig=_grid(18),
    sigma_encoder_network=_mlp(3, 128), sigma_decoder_network=_mlp(3, 128),
    signal_network=dict(_mlp(3, 512), otype="CutlassMLP"),
)
SIMU_MODEL = dict(MESHRIR_MODEL, dir_encoding_sig=_grid(18), signal_output_dim=1600)  # avr_simu.yml model block
RAF_MODEL = dict(  # config_files/avr_raf_furnished.yml:37-100
    signal_output_dim=1600, leaky_relu=0.03,
    pos_encoding_sigma=_grid(18), pos_encoding_sig=_grid(18), dir_encoding_sig=_grid(18),
    tx_pos_encoding_sigma=_grid(18), tx_pos_encoding_sig=_grid(18), tx_dir_encoding_sig=_grid(18),
    sigma_encoder_network=_mlp(3, 128), sigma_decoder_network=_mlp(1, 128),
    signal_network=dict(_mlp(4, 512), otype="CutlassMLP"),
)
