"""When each DDP gradient bucket becomes ready, relative to the backward pass
(verdict r03 item 8; avr_runner_ddp.py:98).

Two ranks on cuda:0 over gloo (the test box has one GPU), the config-4
per-rank shape (4 RAF-Empty poses, AVRModel_complex with the RAF widths) in
the bench's ddp-train setup.  A DDP comm hook records a HIP event on the
current stream when a bucket is handed to the all-reduce; the events are
read back against events at the start and end of backward, so the position
of each bucket in the GPU timeline of backward is measured, not its host
issue time.  The hook communicates nothing (it returns the bucket as is):
over gloo a real all-reduce blocks the autograd thread and stretches the
timeline, so the run measures when each bucket becomes READY in a
compute-only backward; what RCCL then costs is estimated from the bytes.
Prints one JSON line per step from rank 0 and a summary.

    python tools/ddp_buckets.py [--steps 4]
"""
from __future__ import annotations

import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, steps, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from avr_amd import AVRRender
    from avr_amd.criterion import Criterion
    from avr_amd.model import AVRModel_complex
    from avr_amd.parallel import ddp
    from avr_amd.workloads import RAF_MODEL, WORKLOADS

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = WORKLOADS["c4_raf_empty_b4_per_gpu"]
    torch.manual_seed(0)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=w.T), mlp_dtype=torch.float16).to(dev)
    r = AVRRender(model, **w.render).to(dev)
    net = ddp(r, dev)
    names = {p.data_ptr(): n for n, p in r.named_parameters()}
    log = []

    def hook(state, bucket):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        log.append((bucket.index(), bucket.buffer().numel() * 4,
                    sorted({names.get(p.data_ptr(), "?").split(".")[1] if "." in names.get(p.data_ptr(), "?")
                            else names.get(p.data_ptr(), "?") for p in bucket.parameters()}), ev))
        fut = torch.futures.Future()
        fut.set_result(bucket.buffer())
        return fut

    net.register_comm_hook(None, hook)
    crit = Criterion(dict(spec_loss_weight=1, amplitude_loss_weight=1, angle_loss_weight=1, time_loss_weight=20,
                          energy_loss_weight=3, multistft_loss_weight=2), w.render)
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    B, T = w.batch, w.T
    ro = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=dev, generator=g) * 4 - 2
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=dev, generator=g), dim=-1)
    tt = torch.arange(T, device=dev)
    tgt = torch.fft.rfft(torch.randn(B, T, device=dev, generator=g) * torch.exp(-tt / (0.15 * T)) * 0.05)
    res = []
    for step in range(steps):
        log.clear()
        out = net(ro, tx, dtx)
        losses = crit(out, tgt)
        total = losses[0]
        for x in losses[1:8]:
            total = total + x
        net.zero_grad(set_to_none=True)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        total.backward()
        e1.record()
        torch.cuda.synchronize()
        bw = e0.elapsed_time(e1)
        buckets = [{"index": i, "bytes": nb, "modules": mods, "ready_ms": e0.elapsed_time(ev),
                    "ready_frac": e0.elapsed_time(ev) / bw} for i, nb, mods, ev in log]
        res.append({"step": step, "backward_ms": bw, "buckets": buckets})
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    for r in res:
        print(json.dumps(r), flush=True)
    last = res[-1]
    tail = [b for b in last["buckets"] if b["ready_frac"] > 0.9]
    print(json.dumps({"summary": "buckets ready in the last 10% of backward",
                      "bytes": sum(b["bytes"] for b in tail),
                      "total_bytes": sum(b["bytes"] for b in last["buckets"]),
                      "modules": sorted({m for b in tail for m in b["modules"]})}), flush=True)


if __name__ == "__main__":
    main()
