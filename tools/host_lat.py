"""Host/GPU timeline of the serial IR render (bench.py's latency loop: graph
replay, host poses, synchronize per pose).  Records CLOCK_MONOTONIC stamps
around each phase of the host loop; run under rocprofv3 --kernel-trace and
`--report <kernel_trace.csv> <stamps.json>` lines the stamps up with the
kernels (the tracer's timestamps are CLOCK_MONOTONIC too).

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/host_lat.py OUT.json
    python tools/host_lat.py --report DIR/run_kernel_trace.csv OUT.json
"""
import csv
import json
import os
import statistics as st
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(out):
    import torch

    sys.path.insert(0, ROOT)
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
    P = 16
    ro = torch.rand(P, B, 3, generator=torch.Generator().manual_seed(1)) * 4 - 2
    tx = torch.rand(P, B, 3, generator=torch.Generator().manual_seed(2)) * 4 - 2
    r = AVRRender(Stub(attn, sig), **w.render)
    gr = GraphedRender(r, ring=12)
    ns = time.monotonic_ns
    stamps = []
    with torch.no_grad():
        for i in range(30):
            gr.render_ir(ro[i % P], tx[i % P])
        torch.cuda.synchronize()
        for i in range(60):
            t0 = ns()
            gr.render_ir(ro[i % P], tx[i % P])
            t1 = ns()
            torch.cuda.synchronize()
            t2 = ns()
            stamps.append((t0, t1, t2))
    d = [((b - a) / 1e3, (c - b) / 1e3) for a, b, c in stamps]
    print(f"host issue {st.median(x for x, _ in d):.1f} us, wait {st.median(y for _, y in d):.1f} us, "
          f"per pose {st.median(x + y for x, y in d):.1f} us", flush=True)
    json.dump(stamps, open(out, "w"))


def report(trace, stamps_path):
    stamps = json.load(open(stamps_path))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:24])
                for r in csv.DictReader(open(trace)))
    rows = []
    for t0, t1, t2 in stamps:
        inside = [k for k in ks if t0 <= k[0] <= t2]
        if not inside:
            continue
        first, last = inside[0], max(k[1] for k in inside)
        rows.append(((t1 - t0) / 1e3, (first[0] - t0) / 1e3, (first[0] - t1) / 1e3, (last - first[0]) / 1e3,
                     (t2 - last) / 1e3, (t2 - t0) / 1e3, len(inside)))
    if not rows:
        print("no kernels inside the host stamps: clocks differ")
        return
    names = ["host issue", "issue start -> 1st kernel", "issue end -> 1st kernel", "kernels span",
             "last kernel end -> sync returns", "per pose", "kernels"]
    for i, n in enumerate(names):
        print(f"  {n:34s} {st.median(r[i] for r in rows):8.1f}")


if __name__ == "__main__" and sys.argv[1] != "--breakdown":
    if sys.argv[1] == "--report":
        report(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])


def breakdown():
    """Host cost of each step GraphedRender.render_ir takes for a host pose
    (medians over 2000 calls each, GPU work not waited for)."""
    import ctypes
    import timeit

    import torch

    sys.path.insert(0, ROOT)
    from avr_amd import AVRRender, _lib
    from avr_amd.graph import PinnedHostBuffer
    from avr_amd.workloads import WORKLOADS

    dev = torch.device("cuda", 0)
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    r = AVRRender(None, **w.render)
    ro = torch.rand(1, 3)
    buf = PinnedHostBuffer(64)
    jit = buf.host[9:9 + w.render["n_azi"] + w.render["n_ele"]]
    ev = torch.cuda.Event()
    ev.record()
    torch.cuda.synchronize()
    steps = {
        "_device": lambda: r._device(ro),
        "key": lambda: (1, True, ro.is_cuda, dev, tuple(p.data_ptr() for p in r.parameters())),
        "event.query": lambda: ev.query(),
        "torch.rand(out=)": lambda: torch.rand(jit.numel(), out=jit),
        "memmove x2": lambda: (ctypes.memmove(buf._h, ro.data_ptr(), 12), ctypes.memmove(buf._h + 12, ro.data_ptr(), 12)),
        "raw stream": lambda: torch._C._cuda_getCurrentRawStream(0),
        "_lib.call(avr_last_error)": lambda: _lib.load().avr_last_error(),
        "event.record": lambda: ev.record(),
    }
    for name, fn in steps.items():
        t = min(timeit.repeat(fn, number=2000, repeat=5)) / 2000 * 1e6
        print(f"  {name:28s} {t:6.2f} us", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--breakdown":
    breakdown()
