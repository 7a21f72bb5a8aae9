"""The MLP backward's pieces at the shapes one training step uses.

Records the (N, M, K) of every weight-gradient call of one config-3/4
training step (tools/bench_train.py's model), then times each distinct shape
alone with HIP events: the ReLU mask (threshold_backward), the data gradient
(g @ W, hipBLASLt) and the weight gradient (avr_linear_wgrad + finalize),
with the HBM bytes each must move.

    python tools/bench_wgrad.py [--workload c3_raf_furnished_b4] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, model as M  # noqa: E402
from avr_amd.model import AVRModel_complex  # noqa: E402
from avr_amd.training import TrainStep  # noqa: E402
from avr_amd.workloads import RAF_MODEL, WORKLOADS  # noqa: E402


def time_us(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tuned", default=None, help="TunableOp results file: time the data gradients' "
                    "GEMMs with it (tuning off)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    B = w.batch
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=dev, generator=g), dim=-1)
    net = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=w.T), mlp_dtype=torch.bfloat16).to(dev)
    r = AVRRender(net, **w.render).to(dev)
    ts = TrainStep(r, dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5, spec_loss_weight=1,
                            amplitude_loss_weight=1, angle_loss_weight=1, time_loss_weight=20,
                            energy_loss_weight=3, multistft_loss_weight=2), w.render)
    tt = torch.arange(w.T, device=dev)
    ir = torch.randn(B, w.T, device=dev, generator=g) * torch.exp(-tt / (0.15 * w.T)) * 0.05
    target = torch.fft.rfft(ir)

    shapes = []
    orig = M._wgrad

    def rec(gy, x):
        shapes.append((gy.size(0), gy.size(1), x.size(1), M._hip_wgrad_ok(gy, x)))
        return orig(gy, x)

    M._wgrad = rec
    ts(target, ro, tx, dtx)
    torch.cuda.synchronize()
    M._wgrad = orig

    out = []
    for (N, Mo, K, hip) in sorted(set(shapes), key=lambda s: -s[1] * s[2]):
        gy = torch.randn(N, Mo, device=dev, generator=g).to(torch.bfloat16)
        y = torch.relu(torch.randn(N, Mo, device=dev, generator=g)).to(torch.bfloat16)
        x = torch.relu(torch.randn(N, K, device=dev, generator=g)).to(torch.bfloat16)
        wt = (torch.randn(Mo, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
        gm = torch.ops.aten.threshold_backward(gy, y, 0)
        t_mask = time_us(lambda: torch.ops.aten.threshold_backward(gy, y, 0), args.iters)
        t_dgrad = time_us(lambda: gm @ wt, args.iters)
        t_dgrad_tuned = None
        if args.tuned:
            import torch.cuda.tunable as tun
            tun.tuning_enable(False)
            tun.record_untuned_enable(False)
            tun.enable(True)
            tun.read_file(args.tuned)
            t_dgrad_tuned = time_us(lambda: gm @ wt, args.iters)
            tun.enable(False)
        t_wgrad = time_us(lambda: M._wgrad(gm, x), args.iters)
        t_fused = None
        if Mo == 512 and K == 512:  # (g W) masked by the input activation in one launch
            xm = torch.relu(torch.randn(N, K, device=dev, generator=g)).to(torch.bfloat16)
            t_fused = time_us(lambda: M._dgrad512_masked(gm, wt, xm), args.iters)
        out.append(dict(N=N, M=Mo, K=K, hip=hip, calls=shapes.count((N, Mo, K, hip)),
                        mask_us=t_mask, mask_GBps=3 * N * Mo * 2 / t_mask / 1e3,
                        dgrad_us=t_dgrad, dgrad_GBps=(N * Mo + N * K) * 2 / t_dgrad / 1e3,
                        wgrad_us=t_wgrad, wgrad_GBps=(N * Mo + N * K) * 2 / t_wgrad / 1e3,
                        wgrad_TFs=2 * N * Mo * K / t_wgrad / 1e6,
                        fused_dgrad_mask_us=t_fused, dgrad_tuned_us=t_dgrad_tuned))
        print(json.dumps(out[-1]), flush=True)
    tot = {k: sum(o[k] * o["calls"] for o in out) for k in ("mask_us", "dgrad_us", "wgrad_us")}
    print(json.dumps(dict(workload=w.name, per_step_us=tot)))


if __name__ == "__main__":
    main()
