"""Golden vectors for the training criterion from the REAL reference
`utils/criterion.py` (build container only; /root/reference is absent on the
GPU box).

auraloss (the reference's MR-STFT dependency) is not installed.  Its import
is satisfied by a placeholder module whose `MultiResolutionSTFTLoss` returns
NaN: no stored value depends on it (the MR-STFT term stays "parity
unpinned").  Every other term -- spectral (real/imag L1),
amplitude, angle, time, energy decay, and the DAS regression / cross-entropy
terms (criterion.py:69-122) -- runs the reference's own code, and so does
the gradient of their weighted sum w.r.t. the predicted spectrum (autograd
through the reference).  The repo's CPU restatement
(oracle/criterion_oracle.py) must agree with every stored value before a
fixture is written, which is what pins it.

Fixtures hold data only: seeds, shapes, weights, expected losses and
gradients (tests regenerate the inputs from the seeds).

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_criterion_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "criterion")

sys.path.insert(0, os.path.join(REPO, "tests"))
from criterion_cases import CASES, RENDER, spectra  # noqa: E402
from oracle import criterion_oracle as co  # noqa: E402

TERMS = ("spec", "amplitude", "angle", "time", "energy")


def _reference_criterion():
    class _NoMRSTFT(torch.nn.Module):
        """auraloss is absent: the term it computes is never stored."""

        def __init__(self, *a, **k):
            super().__init__()

        def forward(self, x, y):
            return torch.tensor(float("nan"))

    aura = types.ModuleType("auraloss")
    aura.freq = types.SimpleNamespace(MultiResolutionSTFTLoss=_NoMRSTFT)
    sys.modules["auraloss"] = aura
    sys.path.insert(0, REF)
    from utils.criterion import Criterion  # noqa: E402  (the reference's file)

    return Criterion


def main():
    Criterion = _reference_criterion()
    torch.set_num_threads(8)
    for name, B, F, weights, seed in CASES:
        pred, ori = spectra(B, F, seed)
        cfg = dict(weights)
        ref = Criterion(cfg, RENDER)
        p = pred.clone().requires_grad_(True)
        out = ref(p, ori)
        out = [x.detach() if i >= 8 else x for i, x in enumerate(out)]
        losses = [out[i] for i in range(5)] + [out[6], out[7]]
        total = sum(losses)  # every term but the MR-STFT one
        total.backward()
        z = {
            "meta": json.dumps(dict(name=name, B=B, F=F, seed=seed, weights=cfg, render=RENDER,
                                    terms=list(TERMS) + ["das_reg", "das_ce"],
                                    source="utils/criterion.py (reference), MR-STFT not stored")),
            "losses": np.array([float(x.detach()) for x in losses], np.float64),
            "ori_time": out[8].detach().numpy().astype(np.float32),
            "pred_time": out[9].detach().numpy().astype(np.float32),
            "grad": torch.view_as_real(p.grad).numpy().astype(np.float32),
        }
        # pin the repo's restatement to the reference on the same inputs
        q = pred.clone().requires_grad_(True)
        o = co.criterion(q, ori, cfg)
        mine = [o[i] for i in range(5)]
        if cfg.get("das_reg_loss_weight", 0) > 0 or cfg.get("das_ce_loss_weight", 0) > 0:
            mine += list(co.das_losses(q, ori, RENDER["fs"], RENDER["speed"],
                                       cfg.get("das_reg_loss_weight", 0.0), cfg.get("das_ce_loss_weight", 0.0),
                                       cfg.get("beta", 100.0)))
        else:
            mine += [torch.tensor(0.0), torch.tensor(0.0)]
        sum(mine).backward()
        for i, (a, b) in enumerate(zip(mine, z["losses"])):
            if abs(float(a) - b) > 1e-5 * abs(b) + 1e-8:
                raise SystemExit(f"{name}: oracle term {i} {float(a)} != reference {b}")
        g = torch.view_as_real(q.grad).numpy()
        err = np.linalg.norm(g - z["grad"]) / max(np.linalg.norm(z["grad"]), 1e-30)
        if err > 1e-5:
            raise SystemExit(f"{name}: oracle gradient rel err {err}")
        np.savez_compressed(os.path.join(OUT, f"crit_{name}.npz"), **z)
        print(f"crit_{name}: losses {np.array2string(z['losses'], precision=5)} oracle grad err {err:.1e}")


if __name__ == "__main__":
    main()
