"""Interleaved timing of exact-head item shapes (16-bit h, K = 512; config 2
by default, --workload for others, --shard-of N for one rank's ray shard)
with the shape-probe library (`make -C avr_amd/csrc shapes`,
csrc/probe.h): the kernel alone, HIP events around each launch of the full
fused render, rounds interleaved so clock drift hits every shape alike.

    python tools/ab_shapes.py [--shapes 128,256/32,256/64] [--rounds 4]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from avr_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("AVR_AB_LIB") or os.path.join(ROOT, "tools", "_lib", "libavr_shapes.so")
from avr_amd import AVRRender  # noqa: E402
from avr_amd.workloads import WORKLOADS  # noqa: E402


def set_shape(sh):
    # "256/64p": static priority for the second half of the waves, "256/64n":
    # none (AVR_EXACT_PRIO_PROBE; the library's default is on for 8-wave items)
    if sh[-1] in "pn":
        os.environ["AVR_EXACT_PRIO_PROBE"] = "1" if sh[-1] == "p" else "0"
        sh = sh[:-1]
    else:
        os.environ.pop("AVR_EXACT_PRIO_PROBE", None)
    rays, _, tt = sh.partition("/")
    os.environ["AVR_EXACT_RAYS_PROBE"] = rays
    os.environ["AVR_EXACT_TT_PROBE"] = tt or "32"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="128,256/32,256/64")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--workload", default="c2_meshrir_1024x256x512")
    ap.add_argument("--shard-of", type=int, default=1, help="render rank 0's ray shard of an N-rank split")
    args = ap.parse_args()
    dtype = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    w = WORKLOADS[args.workload]
    B, R, S, T, K = w.batch, w.n_rays, w.n_samples, w.T, 512
    from avr_amd.parallel import shard_range
    r0, r1 = shard_range(R, 0, max(1, args.shard_of))
    R = r1 - r0
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(19)
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    h = torch.relu(torch.randn(B, R * S, K, device=dev, generator=g)).to(dtype)
    W = torch.randn(T, K, device=dev, generator=g) / K ** 0.5
    r = AVRRender(None, **w.render)
    if args.shard_of > 1:
        r.ray_range = (r0, r1)
    torch.manual_seed(5)
    _, _, _, _, geom = r.sample(ro, tx)
    shapes = args.shapes.split(",")
    res = {s: [] for s in shapes}
    ref = None
    with torch.no_grad():
        for s in shapes:  # warm every shape; results must agree bit for bit
            set_shape(s)
            out = r.render_from_hidden(attn, h, W, dtype, geom)
            if ref is None:
                ref = out.clone()
            print(s, "equal to", shapes[0], bool(torch.equal(out, ref)), flush=True)
        for _ in range(args.rounds):
            for s in shapes:
                set_shape(s)
                for _ in range(3):
                    r.render_from_hidden(attn, h, W, dtype, geom)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    r.render_from_hidden(attn, h, W, dtype, geom)
                e1.record()
                e1.synchronize()
                res[s].append(e0.elapsed_time(e1) / args.iters * 1e3)
    for s in shapes:
        v = sorted(res[s])
        print(f"shape {s}: fused render {v[len(v) // 2]:.1f} us median (min {v[0]:.1f})", flush=True)


if __name__ == "__main__":
    main()
