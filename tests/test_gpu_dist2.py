"""World size 2 on the one GPU of the test box: two processes (gloo backend,
device tensors) each driving the HIP render on cuda:0, so the multi-rank
decomposition runs through the real kernels rather than the CPU oracle:

* ray-sharded inference (RayShardedRender) == the unsharded render, for a
  stub network and for an fp16 AVRModel_complex (the shards take the
  renderer's own path: ray-layout dedup and the exact fused head);
* ray-sharded training: SUM-all-reduced parameter gradients
  (allreduce_grads_sum) == the unsharded render's gradients;
* DDP over pose shards (avr_runner_ddp.py:37-46,98): gradients after the
  bucketed all-reduce == the mean of the per-pose gradients of a replica, and
  a TrainStep keeps the ranks' weights identical.

RCCL itself needs one GPU per rank, so its N-rank runs belong to the driver's
scaling bench (bench.py --mode ray-shard / ddp-train); tests/test_gpu_dist.py
runs RCCL at world size 1."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        from avr_amd import AVRRender
        from avr_amd.model import AVRModel_complex
        from avr_amd.parallel import RayShardedRender, allreduce_grads_sum, ddp, shard_range
        from avr_amd.training import TrainStep
        from avr_amd.workloads import RAF, RAF_MODEL, WORKLOADS, make_inputs

        # 1. ray-sharded inference through the HIP path
        w = WORKLOADS["c1_meshrir_plumbing"]
        inp = make_inputs(w, 1)
        R, S, T = w.n_rays, w.n_samples, w.T
        attn = torch.from_numpy(inp["attn"]).to(dev)
        sig = torch.from_numpy(inp["signal"]).to(dev)

        class ShardStub(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.r = None

            def forward(self, pts, view, tx, dir_tx=None):
                r0, r1 = self.r.ray_range or (0, R)
                assert pts.size(1) == (r1 - r0) * S
                return attn[:, r0 * S:r1 * S], sig[:, r0 * S:r1 * S]

        stub = ShardStub()
        rr = AVRRender(stub, **w.render)
        stub.r = rr
        ro = torch.from_numpy(inp["rays_o"]).to(dev)
        txp = torch.from_numpy(inp["position_tx"]).to(dev)
        with torch.no_grad():
            torch.manual_seed(1)
            full = rr(ro, txp)
            torch.manual_seed(1)
            shd = RayShardedRender(rr)(ro, txp)
        res["infer_rel"] = _rel(shd, full)

        # 1b. ray shards of a 16-bit network go through the renderer's own
        # path: the shard's ray layout reaches the network (per-ray / per-pose
        # encodings once) and the exact fused head renders; the all-reduced
        # shards equal the unsharded fused render
        cfg16 = dict(RAF, n_azi=8, n_ele=4, n_samples=16)
        torch.manual_seed(0)
        m16 = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800), mlp_dtype=torch.float16).to(dev)
        seen = []
        orig_fused = m16.forward_fused

        def spy(*a, **k):
            seen.append(k.get("ray_layout"))
            return orig_fused(*a, **k)

        m16.forward_fused = spy
        r16 = AVRRender(m16, **cfg16).to(dev)
        g16 = torch.Generator(device=dev).manual_seed(17)
        rx16 = torch.rand(2, 3, device=dev, generator=g16) * 2 - 1
        tx16 = torch.rand(2, 3, device=dev, generator=g16) * 2 - 1
        dtx16 = torch.nn.functional.normalize(torch.randn(2, 3, device=dev, generator=g16), dim=-1)
        with torch.no_grad():
            torch.manual_seed(4)
            full16 = r16(rx16, tx16, dtx16)
            torch.manual_seed(4)
            shd16 = RayShardedRender(r16)(rx16, tx16, dtx16)
        R16 = 8 * 4 + 2
        r0, r1 = shard_range(R16, rank, world)
        res["fp16_shard_rel"] = _rel(shd16, full16)
        res["fp16_layouts"] = seen == [(2, R16, 16), (2, r1 - r0, 16)]

        # 2. ray-sharded training gradients (SUM over ranks)
        cfg = dict(RAF, n_azi=8, n_ele=4, n_samples=16)

        def model(seed):
            torch.manual_seed(seed)
            m = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800)).to(dev)
            return AVRRender(m, **cfg).to(dev)

        g = torch.Generator(device=dev).manual_seed(7)
        rx = torch.rand(2, 3, device=dev, generator=g) * 2 - 1
        tx = torch.rand(2, 3, device=dev, generator=g) * 2 - 1
        dtx = torch.nn.functional.normalize(torch.randn(2, 3, device=dev, generator=g), dim=-1)
        gout = torch.randn(2, 401, 2, device=dev, generator=g)
        a, b = model(0), model(0)
        torch.manual_seed(3)
        (RayShardedRender(a)(rx, tx, dtx) * gout).sum().backward()
        allreduce_grads_sum(a.parameters())
        torch.manual_seed(3)
        (b(rx, tx, dtx) * gout).sum().backward()
        pb = dict(b.named_parameters())
        res["ray_grad_rel"] = max(_rel(p.grad, pb[n].grad) for n, p in a.named_parameters())

        # 3. DDP over pose shards: grads == mean of the per-pose grads
        c = model(0)
        dd = ddp(c, dev)
        p0, p1 = shard_range(2, rank, world)
        torch.manual_seed(5)
        (dd(rx[p0:p1], tx[p0:p1], dtx[p0:p1]) * gout[p0:p1]).sum().backward()
        ref = model(0)
        acc = {n: torch.zeros_like(p) for n, p in ref.named_parameters()}
        for k in range(2):
            ref.zero_grad(set_to_none=True)
            torch.manual_seed(5)
            (ref(rx[k:k + 1], tx[k:k + 1], dtx[k:k + 1]) * gout[k:k + 1]).sum().backward()
            for n, p in ref.named_parameters():
                acc[n] += p.grad / 2
        res["ddp_grad_rel"] = max(_rel(p.grad, acc[n]) for n, p in c.named_parameters())

        # 4. DDP TrainStep: the ranks' weights stay identical
        ts = TrainStep(ddp(model(0), dev), dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5,
                                                  spec_loss_weight=1, amplitude_loss_weight=1,
                                                  angle_loss_weight=1, time_loss_weight=20,
                                                  energy_loss_weight=3, multistft_loss_weight=2),
                       dict(fs=16000, speed=346.8))
        t = torch.arange(800, device=dev)
        ir = torch.randn(2, 800, device=dev, generator=g) * torch.exp(-t / 120.0) * 0.05
        ori = torch.fft.rfft(ir)
        for _ in range(2):
            out = ts(ori[p0:p1], rx[p0:p1], tx[p0:p1], dtx[p0:p1])
            assert out is not None and torch.isfinite(out[0])
        flat = torch.cat([p.detach().reshape(-1) for p in ts.renderer.module.parameters()])
        other = flat.clone()
        dist.broadcast(other, src=0)
        res["ddp_weights_equal"] = bool(torch.equal(flat, other))
        q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put((rank, {"error": repr(e)}))
        raise
    finally:
        dist.destroy_process_group()


def test_world2_gloo_on_one_gpu_hip_path():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = dict(q.get(timeout=100) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, res in out.items():
        assert "error" not in res, (rank, res)
        assert res["infer_rel"] < 1e-5, res
        assert res["fp16_shard_rel"] < 1e-6, res
        assert res["fp16_layouts"], res
        assert res["ray_grad_rel"] < 1e-3, res
        assert res["ddp_grad_rel"] < 1e-3, res
        assert res["ddp_weights_equal"], res
    for p in procs:
        assert p.exitcode == 0
