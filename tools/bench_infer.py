"""End-to-end inference benchmark: the reference network (AVRModel, MeshRIR
`model:` block, random weights) + the renderer + IR for config 2
(1024 rays x 256 samples, T=1022), with and without the fused signal head
 and with / without the fused sigma networks
(csrc/sigma.hip).  One pose per step, no grad.

    python tools/bench_infer.py [--steps 20] [--mlp-dtype bf16]
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

from avr_amd import AVRRender, spectrum_to_ir  # noqa: E402
from avr_amd.model import AVRModel  # noqa: E402
from avr_amd.options import KernelOptions  # noqa: E402
from avr_amd.options import apply as apply_options  # noqa: E402
from avr_amd.workloads import MESHRIR_MODEL, WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mlp-dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--variants", default="unfused,fused_head_only,fused")
    ap.add_argument("--repeat", type=int, default=1, help="alternate the variants this many times (min reported)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    cfg = dict(MESHRIR_MODEL, signal_output_dim=w.T)
    mlp_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.mlp_dtype]
    model = AVRModel(cfg, mlp_dtype=mlp_dtype).to(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    ro = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(w.batch, 3, device=dev, generator=g) * 4 - 2
    res = {"workload": w.name, "ray_samples_per_pose": w.ray_samples, "mlp_dtype": args.mlp_dtype,
           "network": "AVRModel (avr_meshrir.yml model block, random init)"}
    outs = {}
    # (key, fused signal head, fused sigma networks)
    variants = (("unfused", False, False), ("fused_head_only", True, False), ("fused", True, True))
    for key, fused, fsig in [v for _ in range(args.repeat) for v in variants]:
        if key not in args.variants.split(","):
            continue
        apply_options(model, KernelOptions.from_env(KernelOptions(fused_sigma=fsig)))
        r = AVRRender(model, fused_head=fused, **w.render)

        def step():
            with torch.no_grad():
                return spectrum_to_ir(r(ro, tx))

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        res.setdefault(f"{key}_ms_all", []).append(round(ms, 4))
        ms = min(res[f"{key}_ms_all"])
        res[f"{key}_ms_per_pose"] = ms
        res[f"{key}_ray_samples_per_s"] = w.ray_samples / (ms * 1e-3)
        torch.manual_seed(0)
        outs[key] = out
    if "unfused_ms_per_pose" in res and "fused_ms_per_pose" in res:
        res["speedup"] = res["unfused_ms_per_pose"] / res["fused_ms_per_pose"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
