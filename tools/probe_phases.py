"""Phase clocks of the exact head / linear kernels from the probe build
(tools/_lib/libavr_probe.so, `make -C avr_amd/csrc probe`, csrc/probe.h).

The render runs through the shipped library; the one call under study is
redirected to the probe library, whose kernel records per wave: start and
end (100 MHz real-time clock), the prologue, and shader clocks spent in
compute, DMA waits and barriers.

    python tools/probe_phases.py exact [--iters 5]
    python tools/probe_phases.py linear
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, _lib  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402

# AVR_PROBE_LIB: another probe build (tools/build_var.sh NAME "-DAVR_PHASE_PROBES ...")
PROBE = ctypes.CDLL(os.environ.get("AVR_PROBE_LIB") or os.path.join(ROOT, "tools", "_lib", "libavr_probe.so"))
for name in ("avr_head_fwd_exact", "avr_linear_relu_fwd", "avr_linear_pack_w", "avr_last_error"):
    if hasattr(PROBE, name):
        fn = getattr(PROBE, name)
        fn.restype, fn.argtypes = _lib._SIGS[name]


def summarize(buf, what):
    w = buf.view(-1, 16).cpu().numpy().astype(np.float64)
    w = w[w[:, 1] > 0]
    rt0, t1, t2, t3, dma, bar, comp, rt1 = w[:, :8].T
    marks = w[:, 8:]
    clk = (t3 - t1).sum() / ((rt1 - rt0).sum() / 100e6)  # shader clock (Hz)
    span_us = (rt1.max() - rt0.min()) / 100.0
    life = t3 - t1
    res = {
        "kernel": what, "waves": int(len(w)), "shader_ghz": clk / 1e9, "span_us": span_us,
        "wave_life_us": float(life.mean() / clk * 1e6),
        "frac_prologue": float((t2 - t1).sum() / life.sum()),
        "frac_compute": float(comp.sum() / life.sum()),
        "frac_dma_wait": float(dma.sum() / life.sum()),
        "frac_barrier": float(bar.sum() / life.sum()),
        "prologue_us": float((t2 - t1).mean() / clk * 1e6),
        # prologue marks 8.. (kernel-defined), as us after the start, mean over waves
        "marks_us": [float(((marks[:, k] - t1)[marks[:, k] > 0]).mean() / clk * 1e6) if (marks[:, k] > 0).any()
                     else None for k in range(8)],
        "starts_us_p50_p90_max": [float(np.percentile(rt0 - rt0.min(), q) / 100.0) for q in (50, 90, 100)],
        "ends_us_p10_p50_max": [float(np.percentile(rt1 - rt0.min(), q) / 100.0) for q in (10, 50, 100)],
    }
    print(json.dumps(res), flush=True)


def dump_items(buf, path):
    """Raw per-(item, wave) records of the exact head for offline analysis."""
    w = buf.view(-1, 16).cpu().numpy()
    np.save(path, w[w[:, 1] > 0])


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "exact"
    # phase-skip bitmasks to run (probe build only; results wrong): 1 = no W
    # DMA, 2 = no epilogue, 4 = no row loads (csrc/head_exact.hip)
    skips = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(19)
    buf = torch.zeros(1 << 22, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    if what == "exact":
        assert PROBE.avr_probe_set_exact(ctypes.c_void_p(buf.data_ptr())) == 0
        w = WORKLOADS["c2_meshrir_1024x256x512"]
        B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, 512
        ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
        tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
        attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
        h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(torch.float16)
        W = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
        r = AVRRender(None, **w.render)
        torch.manual_seed(5)
        _, _, _, _, geom = r.sample(ro, tx)
        real_call = _lib.call

        def call(name, *args):
            if name == "avr_head_fwd_exact":
                rc = PROBE.avr_head_fwd_exact(*args)
                if rc:
                    raise RuntimeError(PROBE.avr_last_error().decode())
                return
            real_call(name, *args)

        with torch.no_grad():
            for _ in range(3):
                r.render_from_hidden(attn, h, W, torch.float16, geom)
            _lib.call = call
            import avr_amd.renderer as rr
            rr._lib.call = call
            for sk in skips:
                assert PROBE.avr_probe_set_exact_skip(sk) == 0
                for _ in range(2):
                    buf.zero_()
                    r.render_from_hidden(attn, h, W, torch.float16, geom)
                    torch.cuda.synchronize()
                    summarize(buf, f"exact_head skip={sk}")
                    if os.environ.get("AVR_PROBE_DUMP"):
                        dump_items(buf, os.path.join(os.environ["AVR_PROBE_DUMP"], f"exact_skip{sk}.npy"))
            assert PROBE.avr_probe_set_exact_skip(0) == 0
    else:
        assert PROBE.avr_probe_set_linear(ctypes.c_void_p(buf.data_ptr())) == 0
        M, N, K = 262144, 512, 512
        x = torch.relu(torch.randn(M, K, device=dev, generator=g)).to(torch.float16)
        wt = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.float16)
        wf = torch.empty_like(wt)
        y = torch.empty(M, N, dtype=torch.float16, device=dev)
        assert PROBE.avr_linear_pack_w(N, K, wt.data_ptr(), _lib.DTYPE_F16, wf.data_ptr(), st) == 0
        for _ in range(20):
            PROBE.avr_linear_relu_fwd(M, N, K, x.data_ptr(), wf.data_ptr(), _lib.DTYPE_F16, 1, y.data_ptr(), st)
        for _ in range(3):
            buf.zero_()
            assert PROBE.avr_linear_relu_fwd(M, N, K, x.data_ptr(), wf.data_ptr(), _lib.DTYPE_F16, 1,
                                             y.data_ptr(), st) == 0
            torch.cuda.synchronize()
            summarize(buf, "linear")


if __name__ == "__main__":
    main()
