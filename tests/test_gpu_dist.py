"""The multi-GPU path over RCCL (backend "nccl") on the one GPU of the test
box: a world-size-1 process group, so the collectives run through RCCL on
device tensors (broadcast of the ray jitter, the spectrum all-reduce and its
backward, DDP's bucketed gradient all-reduce of a training step).  The
decomposition across ranks is covered by tests/test_dist_cpu.py (gloo,
world size 2); N-GPU runs belong to the driver's scaling bench."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from avr_amd import AVRRender
from avr_amd.model import AVRModel_complex
from avr_amd.parallel import RayShardedRender, allreduce_spectrum, broadcast_jitter, ddp
from avr_amd.training import TrainStep
from avr_amd.workloads import RAF, RAF_MODEL

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
RAF_TRAIN = dict(lr=2e-4, weight_decay=0, T_max=300000, eta_min=8e-5,
                 spec_loss_weight=1, amplitude_loss_weight=1, angle_loss_weight=1,
                 time_loss_weight=20, energy_loss_weight=3, multistft_loss_weight=2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl():
    torch.cuda.set_device(DEV)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=DEV)
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


def _model(seed):
    torch.manual_seed(seed)
    cfg = dict(RAF, n_azi=8, n_ele=4, n_samples=16)
    model = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800)).to(DEV)
    return AVRRender(model, **cfg).to(DEV)


def _batch():
    B = 2
    g = torch.Generator(device=DEV).manual_seed(7)
    rx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    tx = torch.rand(B, 3, device=DEV, generator=g) * 2 - 1
    dtx = torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
    t = torch.arange(800, device=DEV)
    ir = torch.randn(B, 800, device=DEV, generator=g) * torch.exp(-t / 120.0) * 0.05
    return torch.fft.rfft(ir), rx, tx, dtx


def test_rccl_jitter_broadcast_and_spectrum_allreduce(rccl):
    u = torch.rand(17)
    assert torch.equal(broadcast_jitter(u, None, DEV), u)
    x = torch.randn(2, 129, 2, device=DEV, requires_grad=True)
    y = allreduce_spectrum(x)
    assert torch.equal(y.detach(), x.detach())
    g = torch.randn_like(y)
    y.backward(g)
    assert torch.equal(x.grad, g)  # replicated loss: the all-reduce's backward is the identity


def test_ray_sharded_render_over_rccl_matches_plain_render(rccl):
    r = _model(0)
    _, rx, tx, dtx = _batch()
    with torch.no_grad():
        torch.manual_seed(3)
        ref = r(rx, tx, dtx)
        torch.manual_seed(3)
        out = RayShardedRender(r)(rx, tx, dtx)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-7)


def test_ddp_training_step_over_rccl_equals_single_process(rccl):
    ori, rx, tx, dtx = _batch()
    plain = TrainStep(_model(0), RAF_TRAIN, dict(fs=16000, speed=346.8))
    wrapped = TrainStep(ddp(_model(0), DEV), RAF_TRAIN, dict(fs=16000, speed=346.8))
    for _ in range(2):
        torch.manual_seed(1)
        t0, _ = plain(ori, rx, tx, dtx)
        torch.manual_seed(1)
        t1, _ = wrapped(ori, rx, tx, dtx)
        assert torch.isfinite(t1)
        torch.testing.assert_close(t1, t0, rtol=1e-4, atol=0)  # hash-grid atomics: last-bit run-to-run noise
    # hash-grid backward atomics sum in run-dependent order, and Adam turns a
    # last-bit difference of a near-zero gradient into up to ~lr per step:
    # bound every element by 2 steps of lr and require almost all to agree
    pa = dict(plain.renderer.named_parameters())
    lr = RAF_TRAIN["lr"]
    for n, p in wrapped.renderer.module.named_parameters():
        d = (p.detach() - pa[n].detach()).abs()
        assert float(d.max()) <= 2 * 2 * lr, n
        assert float((d > 1e-6).float().mean()) < 1e-3, n
