"""A/B timing of `avr_ray_pose_bias` (csrc/hashgrid.hip) across library
builds (tools/build_var.sh NAME DEFS hashgrid.hip), config-2 geometry
through AVRModel's own call (model._ray_pose_bias), HIP events, interleaved.

    python tools/xbench_bias.py base=tools/_lib/libvar_hbase.so,v1=tools/_lib/libvar_hv1.so
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from avr_amd import AVRRender, _lib  # noqa: E402
from avr_amd.model import AVRModel, _bias_columns, _ray_pose_bias  # noqa: E402
from avr_amd.workloads import MESHRIR_MODEL, WORKLOADS  # noqa: E402


class _Swap:
    def __init__(self, prod, alt, names):
        self.prod, self.alt, self.names = prod, alt, names
        for n in names:
            fn = getattr(alt, n)
            fn.restype, fn.argtypes = _lib._SIGS[n]
        alt.avr_last_error.restype = ctypes.c_char_p

    def __getattr__(self, name):
        return getattr(self.alt if name in self.names or name == "avr_last_error" else self.prod, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[a.workload]
    model = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=w.T), mlp_dtype=torch.float16).to(dev)
    r = AVRRender(model, **w.render)
    g = torch.Generator(device=dev).manual_seed(4)
    pts, view, tx, _, geom = r.sample(torch.rand(1, 3, device=dev, generator=g) * 4 - 2,
                                      torch.rand(1, 3, device=dev, generator=g) * 4 - 2)
    L = (1, geom["n_rays"], w.n_samples)
    wd, wt = _bias_columns(model._model_signal.layers[0].weight, torch.float16)
    prod = _lib.load()
    libs = [(n, _Swap(prod, ctypes.CDLL(os.path.join(ROOT, p)), ["avr_ray_pose_bias"]))
            for n, p in (i.split("=", 1) for i in a.libs.split(","))]

    def run():
        return _ray_pose_bias(model._dir_encoding, model._tx_encoding, view, tx, wd, wt, L, torch.float16)

    outs, times = {}, {n: [] for n, _ in libs}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    with torch.no_grad():
        for name, lib in libs:
            _lib._lib = lib
            run()
            outs[name] = run().clone()
        for _ in range(a.rounds):
            for name, lib in libs:
                _lib._lib = lib
                for e0, e1 in ev:
                    e0.record()
                    run()
                    e1.record()
                torch.cuda.synchronize()
                times[name] += [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
    _lib._lib = prod
    ref = outs[libs[0][0]]
    for name, _ in libs:
        t = sorted(times[name])
        print(json.dumps({"lib": name, "workload": a.workload, "median_us": t[len(t) // 2], "min_us": t[0],
                          "bitwise_equal_to_" + libs[0][0]: bool(torch.equal(outs[name], ref))}), flush=True)


if __name__ == "__main__":
    main()
