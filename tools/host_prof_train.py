"""Host-side profile of the training step (cProfile over K steps issued
back to back, one sync at the end): where the Python/ctypes time goes.

    python tools/host_prof_train.py [--workload c3_raf_furnished_b4] [--steps 20]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender  # noqa: E402
from avr_amd.model import AVRModel_complex  # noqa: E402
from avr_amd.training import TrainStep  # noqa: E402
from avr_amd.workloads import RAF_MODEL, WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=w.T), mlp_dtype=torch.bfloat16).to(dev)
    r = AVRRender(model, **w.render).to(dev)
    cfg = dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5, spec_loss_weight=1, amplitude_loss_weight=1,
               angle_loss_weight=1, time_loss_weight=20, energy_loss_weight=3, multistft_loss_weight=2)
    ts = TrainStep(r, cfg, w.render, nan_check=False)
    g = torch.Generator(device=dev).manual_seed(1)
    ro = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    dtx = torch.nn.functional.normalize(torch.randn(w.batch, 3, device=dev, generator=g), dim=-1)
    tgt = torch.fft.rfft(torch.randn(w.batch, w.T, device=dev, generator=g) * 0.05)
    for _ in range(5):
        ts(tgt, ro, tx, dtx)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        ts(tgt, ro, tx, dtx)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    print(s.getvalue())


if __name__ == "__main__":
    main()
