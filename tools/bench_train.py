"""Training-step benchmark for BASELINE configs[2]/[3] (RAF, batch 4 per GPU).

Two numbers, both fwd+bwd:
  * render core only: stub network outputs resident in HBM, grads to attn and
    signal (the hot path's backward);
  * full step (avr_amd.training.TrainStep, avr_runner.py:160-200):
    AVRModel_complex (6 HIP hash grids + MLPs) -> renderer -> the reference
    criterion on the GPU (HIP: spectral, time, energy-decay, multi-resolution
    STFT) -> backward -> clip_grad_norm_ + NaN/Inf zeroing (one HIP launch)
    -> Adam -> CosineAnnealingLR.  `--loss l1` swaps the criterion for a
    plain L1 on the spectrum (the round-1 stand-in, for comparison);
    `--nan-check` adds the reference's per-step host sync on the energy loss.

    python tools/bench_train.py [--workload c3_raf_furnished_b4] [--steps 20] [--mlp-dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender  # noqa: E402
from avr_amd.model import AVRModel_complex  # noqa: E402
from avr_amd.options import KernelOptions  # noqa: E402
from avr_amd.training import TrainStep  # noqa: E402
from avr_amd.workloads import RAF_MODEL, WORKLOADS  # noqa: E402


class Stub(torch.nn.Module):
    def __init__(self, attn, signal):
        super().__init__()
        self.attn, self.signal = attn, signal

    def forward(self, pts, view, tx, dir_tx=None):
        return self.attn, self.signal


def timeit(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def gpu_and_host_ms(fn, steps, spin_cycles=int(4e8)):
    """(GPU ms per step, host issue ms per step, spin ms): the loop is issued
    behind a spin kernel, so the events around it time the GPU's own work
    back to back while the host's issue time is measured apart.  The GPU
    figure is valid when the whole issue took less than the spin."""
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s0.record()
    torch.cuda._sleep(spin_cycles)
    s1.record()
    torch.cuda.synchronize()
    spin_ms = s0.elapsed_time(s1)
    torch.cuda._sleep(spin_cycles)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    host_total = (time.perf_counter() - t0) * 1e3
    e1.record()
    torch.cuda.synchronize()
    gpu = e0.elapsed_time(e1) / steps if host_total < 0.8 * spin_ms else None
    return gpu, host_total / steps, spin_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mlp-dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--core-only", action="store_true")
    ap.add_argument("--no-fused", action="store_true", help="materialise the signal (no fused head)")
    ap.add_argument("--foreach-adam", action="store_true", help="torch's default (foreach) Adam")
    ap.add_argument("--torch-adam", action="store_true", help="torch's fused Adam + avr_scale_sanitize "
                    "instead of the one-pass avr_adam_step")
    ap.add_argument("--profile", action="store_true", help="torch.profiler table of a few steps")
    ap.add_argument("--loss", default="criterion", choices=["criterion", "l1"])
    ap.add_argument("--nan-check", action="store_true", help="reference's per-step isnan().item()")
    ap.add_argument("--sync-debug", action="store_true", help="report the torch ops of one step that "
                    "synchronise with the device (torch.cuda.set_sync_debug_mode), with their stacks")
    ap.add_argument("--torch-norm", action="store_true", help="the fused Adam path's clip coefficient by "
                    "torch's foreach norm (the round-5 form) instead of avr_grad_clip_coef")
    ap.add_argument("--torch-total", action="store_true", help="the loss total by seven torch adds "
                    "(avr_runner.py:187 as written) instead of the criterion kernel's own sum")
    args = ap.parse_args()
    if args.torch_total:
        from avr_amd.criterion import Criterion

        def _torch_total(self, pred_sig, ori_sig):
            out = self.forward(pred_sig, ori_sig)
            total = out[0]
            for x in out[1:8]:
                total = total + x
            return out, total
        Criterion.forward_total = _torch_total
    if args.torch_norm:
        from avr_amd import training as _tr
        _tr._native_clip_coef = lambda grads, max_norm, dev: _tr._clip_coef(grads, max_norm)
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=dev, generator=g), dim=-1)
    res = {"workload": w.name, "ray_samples_per_step": w.ray_samples}

    # render core fwd+bwd
    attn = (torch.rand(B, R * S, 1, device=dev, generator=g) * 2).requires_grad_(True)
    sig = (torch.randn(B, R * S, T, device=dev, generator=g) * 0.1).requires_grad_(True)
    rc = AVRRender(Stub(attn, sig), **w.render)
    gout = torch.randn(B, T // 2 + 1, 2, device=dev, generator=g)

    def core():
        attn.grad = None
        sig.grad = None
        out = rc(ro, tx, dtx)
        out.backward(gout)

    t = timeit(core, args.steps, args.warmup)
    res["render_core_fwd_bwd_ms"] = t * 1e3
    res["render_core_ray_samples_per_s"] = w.ray_samples / t
    # algorithmic bytes: read x twice (fwd, bwd), write grad x, attn/grad attn, w/delay
    alg = w.ray_samples * (3 * T * 4 + 4 * 4)
    res["render_core_alg_GBps"] = alg / t / 1e9
    del attn, sig, rc
    if args.core_only:
        print(json.dumps(res))
        return

    # full training step
    mlp_dtype = torch.bfloat16 if args.mlp_dtype == "bf16" else torch.float32
    cfg = dict(RAF_MODEL, signal_output_dim=T)
    model = AVRModel_complex(cfg, mlp_dtype=mlp_dtype, options=KernelOptions.from_env()).to(dev)
    r = AVRRender(model, fused_head=not args.no_fused, **w.render).to(dev)
    # RAF training config (config_files/avr_raf_*.yml:24-40); the same Adam as
    # the reference's torch.optim.Adam, as one fused multi-tensor kernel
    train_cfg = dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5,
                     spec_loss_weight=1, amplitude_loss_weight=1, angle_loss_weight=1,
                     time_loss_weight=20, energy_loss_weight=3, multistft_loss_weight=2)
    ts = TrainStep(r, train_cfg, w.render, fused_adam=not args.foreach_adam,
                   nan_check=args.nan_check, native_adam=not (args.torch_adam or args.foreach_adam))
    # measured-IR-like target spectrum: decaying noise
    tt = torch.arange(T, device=dev)
    ir = torch.randn(B, T, device=dev, generator=g) * torch.exp(-tt / (0.15 * T)) * 0.05
    target_c = torch.fft.rfft(ir)
    target = torch.view_as_real(target_c).contiguous()
    opt = ts.optimizer

    def train_step():
        if args.loss == "criterion":
            ts(target_c, ro, tx, dtx)
            return
        out = r(ro, tx, dtx)
        loss = (out - target).abs().mean()
        opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(r.parameters(), max_norm=1)
        opt.step()

    t = timeit(train_step, args.steps, args.warmup)
    if args.sync_debug:
        import traceback
        import warnings

        def show(message, category, filename, lineno, file=None, line=None):
            print(f"SYNC: {message}", file=sys.stderr)
            print("".join(traceback.format_stack(limit=14)[:-2]), file=sys.stderr)

        warnings.showwarning = show
        warnings.simplefilter("always")
        torch.cuda.set_sync_debug_mode("warn")
        train_step()
        torch.cuda.set_sync_debug_mode("default")
        torch.cuda.synchronize()
    if args.profile:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                train_step()
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=40), file=sys.stderr)
    res["train_step_ms"] = t * 1e3
    gpu, host, spin = gpu_and_host_ms(train_step, args.steps)
    res["train_step_gpu_ms"] = gpu  # the steps' GPU work back to back (None: issue outlasted the spin)
    res["train_step_host_issue_ms"] = host
    res["spin_ms"] = spin
    res["train_ray_samples_per_s"] = w.ray_samples / t
    res["mlp_dtype"] = args.mlp_dtype
    res["fused_head"] = not args.no_fused
    res["adam"] = "foreach" if args.foreach_adam else ("avr_adam_step" if ts.native_adam else "fused")
    res["loss"] = args.loss
    res["nan_check"] = args.nan_check
    print(json.dumps(res))


if __name__ == "__main__":
    main()
