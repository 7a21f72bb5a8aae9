"""Networks the renderer drives: `AVRModel` (MeshRIR / Simu / Real_env) and
`AVRModel_complex` (RAF), model.py:63-235 and 238-331 of the reference.

Encodings are the HIP hash grid (`avr_amd.encoding`); the MLPs are plain
`nn.Linear(bias=False)` stacks with ReLU (tcnn FullyFusedMLP / CutlassMLP
have no biases), run by PyTorch-ROCm (hipBLASLt GEMMs) so autograd covers
them.  `mlp_dtype` selects the GEMM precision (tcnn runs its MLPs in fp16;
bf16 is the MI355X MFMA-native choice).  The channel-embedding ablations of
AVRModel (model.py:71-181, "injection"/"concat") are outside the hot path
and not provided.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .encoding import HashGridEncoding


class MLP(nn.Module):
    """tcnn.Network(n_in, n_out, {n_neurons, n_hidden_layers, activation ReLU,
    output_activation None}) without biases."""

    def __init__(self, n_in, n_out, cfg, dtype=torch.float32):
        super().__init__()
        width = int(cfg["n_neurons"])
        depth = int(cfg["n_hidden_layers"])
        if cfg.get("activation", "ReLU") != "ReLU":
            raise ValueError("only ReLU MLPs are used by the reference configs")
        dims = [n_in] + [width] * depth + [n_out]
        self.layers = nn.ModuleList(nn.Linear(a, b, bias=False) for a, b in zip(dims[:-1], dims[1:]))
        self.dtype = dtype
        self.n_output_dims = n_out

    def forward(self, x):
        x = x.to(self.dtype)
        for i, lin in enumerate(self.layers):
            x = F.linear(x, lin.weight.to(self.dtype))
            if i + 1 < len(self.layers):
                x = F.relu(x)
        return x


class AVRModel(nn.Module):
    """model.py:63-235 without channel embedding: pos/dir/tx hash grids,
    sigma encoder (-> 128) and decoder (-> 1), signal network (-> T)."""

    def __init__(self, cfg, mlp_dtype=torch.float32, enc_dtype=torch.float16):
        super().__init__()
        self._pos_encoding = HashGridEncoding(3, cfg["pos_encoding_sigma"], dtype=enc_dtype, seed=1)
        self._dir_encoding = HashGridEncoding(3, cfg["dir_encoding_sig"], dtype=enc_dtype, seed=2)
        self._tx_encoding = HashGridEncoding(3, cfg["tx_encoding_sig"], dtype=enc_dtype, seed=3)
        self.signal_output_dim = int(cfg["signal_output_dim"])
        self._model_encoder_sigma = MLP(self._pos_encoding.n_output_dims, 128,
                                        cfg["sigma_encoder_network"], mlp_dtype)
        self._model_decoder_sigma = MLP(128, 1, cfg["sigma_decoder_network"], mlp_dtype)
        sig_in = 128 + self._dir_encoding.n_output_dims + self._tx_encoding.n_output_dims
        self._model_signal = MLP(sig_in, self.signal_output_dim, cfg["signal_network"], mlp_dtype)

    def forward(self, pts, view, tx, ch_idx=None):
        if ch_idx is not None:
            raise NotImplementedError("channel-embedding variants are not provided")
        bs, n = pts.size(0), pts.size(1)
        pos_enc = self._pos_encoding((pts.reshape(-1, 3) + 1) / 2)
        sigma_feat = self._model_encoder_sigma(pos_enc)
        attn = self._model_decoder_sigma(F.relu(sigma_feat))
        dir_enc = self._dir_encoding((view.reshape(-1, 3) + 1) / 2)
        tx_enc = self._tx_encoding((tx.reshape(-1, 3) + 1) / 2)
        dt = sigma_feat.dtype
        base = torch.cat([sigma_feat, dir_enc.to(dt), tx_enc.to(dt)], dim=-1)
        signal = self._model_signal(base)
        attn = torch.abs(F.leaky_relu(attn)).view(bs, n, 1)
        return attn, signal.view(bs, n, self.signal_output_dim)


class AVRModel_complex(nn.Module):  # noqa: N801  (reference name)
    """model.py:238-331: six hash grids (pos/tx for sigma and for signal,
    view and tx orientation), sigma encoder (-> 256) / decoder, signal MLP."""

    def __init__(self, cfg, mlp_dtype=torch.float32, enc_dtype=torch.float32):
        super().__init__()
        self.leaky_relu = cfg["leaky_relu"]
        self.signal_output_dim = int(cfg["signal_output_dim"])
        E = lambda key, seed: HashGridEncoding(3, cfg[key], dtype=enc_dtype, seed=seed)  # noqa: E731
        self._pos_encoding = E("pos_encoding_sigma", 11)
        self._pos_signal_encoding = E("pos_encoding_sig", 12)
        self._tx_pos_encoding = E("tx_pos_encoding_sigma", 13)
        self._tx_pos_signal_encoding = E("tx_pos_encoding_sig", 14)
        self._dir_encoding = E("dir_encoding_sig", 15)
        self._tx_dir_encoding = E("tx_dir_encoding_sig", 16)
        n_in = self._pos_encoding.n_output_dims + self._tx_pos_encoding.n_output_dims
        self._model_encoder_sigma = MLP(n_in, 256, cfg["sigma_encoder_network"], mlp_dtype)
        self._model_decoder_sigma = MLP(256, 1, cfg["sigma_decoder_network"], mlp_dtype)
        n_sig = (256 + self._dir_encoding.n_output_dims + self._tx_dir_encoding.n_output_dims
                 + self._pos_signal_encoding.n_output_dims + self._tx_pos_signal_encoding.n_output_dims)
        self._model_signal = MLP(n_sig, self.signal_output_dim, cfg["signal_network"], mlp_dtype)

    def forward(self, pts, view, tx, tx_view):
        bs, n = pts.size(0), pts.size(1)
        pts = (pts.reshape(-1, 3) + 1) / 2
        view = (view.reshape(-1, 3) + 1) / 2
        tx = (tx.reshape(-1, 3) + 1) / 2
        tx_view = (tx_view.reshape(-1, 3) + 1) / 2
        pos_e = self._pos_encoding(pts)
        txp_e = self._tx_pos_encoding(tx)
        feat = self._model_encoder_sigma(torch.cat([pos_e, txp_e], -1))
        attn = self._model_decoder_sigma(F.relu(feat))
        dt = feat.dtype
        parts = [F.relu(feat), self._dir_encoding(view).to(dt), self._tx_dir_encoding(tx_view).to(dt),
                 self._pos_signal_encoding(pts).to(dt), self._tx_pos_signal_encoding(tx).to(dt)]
        signal = self._model_signal(torch.cat(parts, -1))
        attn = torch.abs(F.leaky_relu(attn, negative_slope=self.leaky_relu)).view(bs, n, 1)
        return attn, signal.reshape(bs, n, self.signal_output_dim)
