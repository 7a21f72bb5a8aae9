"""Run the bf16x3 DFT forms of tools/bf3_repro.sh on the shape that showed
run-to-run differences in round 4 (config 3, AVR_KSPLIT=25: every DFT
workgroup holds one 64-t tile), DESIGN.md §14d.

Per form: the same partials through `avr_dft_phase_fwd` REPEAT times; how
many spectrum partials differ from the first call, which bins (f mod 32)
they fall in, and the relative error against the fp32 form.

    python tools/bf3_repro.py [--repeat 20] [--ksplit 25]
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, _lib  # noqa: E402
from avr_amd.renderer import _ptr, _stream, ctypes_ref, get_tables  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402

FORMS = ["f32", "asm", "noasm", "pin", "nop", "sched"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=20)
    ap.add_argument("--ksplit", type=int, default=25)
    ap.add_argument("--workload", default="c3_raf_furnished_b4")
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    F = T // 2 + 1
    dev = torch.device("cuda", 0)
    r = AVRRender(None, **w.render)
    p = r._params(T, R)
    tables = get_tables(p, dev)
    st = _stream(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    part = torch.randn(1, B, S, T, device=dev, generator=g)
    P = math.ceil(S / 32) * a.ksplit
    ref = None
    for form in FORMS:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_lib", f"libbf3_{form}.so"))
        fn = lib.avr_dft_phase_fwd
        fn.restype, fn.argtypes = _lib._SIGS["avr_dft_phase_fwd"]
        outs = []
        for _ in range(a.repeat):
            spart = torch.full((B, P, F, 2), float("nan"), device=dev)
            rc = fn(ctypes_ref(p), B, _ptr(part), 1, _ptr(tables.pl), _ptr(tables.shift), _ptr(tables.phase),
                    _ptr(tables.twiddle), a.ksplit, _ptr(spart), st)
            assert rc == 0
            outs.append(spart)
        torch.cuda.synchronize()
        first = outs[0]
        diff = torch.zeros(B, P, F, dtype=torch.bool, device=dev)
        for o in outs[1:]:
            diff |= (o != first).any(-1)
        nd = int(diff.sum())
        bins = collections.Counter((torch.nonzero(diff)[:, 2] % 32).tolist()) if nd else {}
        if form == "f32":
            ref = first
        rel = float((first - ref).norm() / ref.norm())
        print(json.dumps({"form": form, "workload": a.workload, "k_split": a.ksplit, "repeats": a.repeat,
                          "partials_differing_between_calls": nd, "of": B * P * F,
                          "bins_mod_32": dict(sorted(bins.items())), "rel_l2_vs_f32": rel,
                          "finite": bool(torch.isfinite(first).all())}), flush=True)


if __name__ == "__main__":
    main()
