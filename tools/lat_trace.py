"""Kernel timeline of the serial IR render (config 2, stub network, host
poses as in bench.py's latency loop): run under rocprofv3 --kernel-trace,
then `python tools/lat_trace.py --report <kernel_trace.csv>` prints, per
pose, every kernel's duration and the idle gap before it, and the medians.

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/lat_trace.py [--eager]
"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(eager):
    import torch

    sys.path.insert(0, ROOT)
    if "--shapes" in sys.argv:  # the shape-probe library (make -C avr_amd/csrc shapes): AVR_*_PROBE switches
        from avr_amd import _lib

        _lib.LIB_PATH = os.path.join(ROOT, "tools", "_lib", "libavr_shapes.so")
    from avr_amd import AVRRender
    from avr_amd.graph import GraphedRender
    from avr_amd.workloads import WORKLOADS

    class Stub(torch.nn.Module):
        draws_no_device_rng = True

        def __init__(self, a, s):
            super().__init__()
            self.a, self.s = a, s

        def forward(self, *args, **kw):
            return self.a, self.s

    dev = torch.device("cuda", 0)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    g = torch.Generator(device=dev).manual_seed(0)
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    attn = torch.rand(B, R * S, 1, device=dev, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=dev, generator=g) * 0.1
    ro = torch.rand(B, 3, generator=torch.Generator().manual_seed(1)) * 4 - 2
    tx = torch.rand(B, 3, generator=torch.Generator().manual_seed(2)) * 4 - 2
    r = AVRRender(Stub(attn, sig), **w.render)
    fn = (lambda: r.render_ir(ro.to(dev), tx.to(dev))) if eager else GraphedRender(r).render_ir
    with torch.no_grad():
        for _ in range(8):
            fn(ro, tx) if not eager else fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 40
        for _ in range(n):
            fn(ro, tx) if not eager else fn()
            torch.cuda.synchronize()
        print(f"latency_ms {(time.perf_counter() - t0) * 1e3 / n:.4f}", flush=True)


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0].split("<")[0][:28]


def report(path, last=10):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    firsts = [i for i, k in enumerate(ks) if k[2].startswith("sample_rays")]
    poses = []
    for a, b in zip(firsts[-last - 1:-1], firsts[-last:]):
        poses.append(ks[a:b])
    per = {}
    for p in poses:
        prev_end = None
        line = []
        for s, e, n in p:
            gap = 0.0 if prev_end is None else (s - prev_end) / 1e3
            per.setdefault(n, []).append(((e - s) / 1e3, gap))
            line.append(f"{n}:{(e - s) / 1e3:.1f}(+{gap:.1f})")
            prev_end = e
        span = (p[-1][1] - p[0][0]) / 1e3
        print(f"span {span:7.1f} us | " + " ".join(line))
    import statistics as st
    print("median per kernel: duration, gap before")
    for n, v in per.items():
        print(f"  {n:28s} {st.median(x for x, _ in v):7.2f} {st.median(g for _, g in v):7.2f}")
    spans = [(p[-1][1] - p[0][0]) / 1e3 for p in poses]
    between = [(b[0][0] - a[-1][1]) / 1e3 for a, b in zip(poses, poses[1:])]
    print(f"median span {st.median(spans):.1f} us, median idle between poses {st.median(between):.1f} us")


if __name__ == "__main__":
    if "--report" in sys.argv:
        report(sys.argv[sys.argv.index("--report") + 1])
    else:
        run("--eager" in sys.argv)
