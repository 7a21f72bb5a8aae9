"""GraphedRender (HIP-graph replay of the inference render) against the eager
render on the same seeded jitter: bit-identical spectrum and IR, new poses
and jitter picked up on every replay."""
import pytest
import torch

from avr_amd import AVRRender
from avr_amd.graph import GraphedRender
from avr_amd.workloads import WORKLOADS

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class Stub(torch.nn.Module):
    draws_no_device_rng = True

    def __init__(self, a, s):
        super().__init__()
        self.a, self.s = a, s

    def forward(self, *args, **kw):
        return self.a, self.s


class StubUndeclared(Stub):
    """A network that does not declare itself free of device RNG."""
    draws_no_device_rng = False


@pytest.mark.parametrize("net", [Stub, StubUndeclared])
@pytest.mark.parametrize("host_pose", [False, True])
@pytest.mark.parametrize("name", ["c2_meshrir_1024x256x512", "c3_raf_furnished_b4"])
def test_graph_replay_equals_eager(name, host_pose, net):
    """Device poses (copied into the graph's tensors) and host poses (staged
    in the pinned buffer, published by the sampling kernel) both replay the
    eager render bit for bit, launched by avr_graph_launch (declared
    RNG-free network) or by torch's CUDAGraph.replay (any other)."""
    w = WORKLOADS[name]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(1)
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=DEV, generator=g) * 0.1
    r = AVRRender(net(attn, sig), **w.render)
    gr = GraphedRender(r)
    for k in range(5):  # captures (ring of 3), then replays with new poses and jitter
        ro = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
        tx = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
        dtx = (torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
               if w.with_dir_tx else None)
        with torch.no_grad():
            torch.manual_seed(10 + k)
            out_e, ir_e = r.render_ir(ro, tx, dtx)
            torch.manual_seed(10 + k)
            if host_pose:
                out_g, ir_g = gr.render_ir(ro.cpu(), tx.cpu(), None if dtx is None else dtx.cpu())
            else:
                out_g, ir_g = gr.render_ir(ro, tx, dtx)
            torch.cuda.synchronize()
        assert torch.equal(out_g, out_e), k
        assert torch.equal(ir_g, ir_e), k
    assert len(gr._graphs) == 1
    inst = next(iter(gr._graphs.values()))[0][0]
    assert (inst.exec is not None) == (net is Stub)


def test_graph_ring_pipelined_replays():
    """Replays issued back to back without a host sync: each ring instance
    is reused only after its previous replay ran, so every render keeps its
    own host pose and jitter draw (compared with eager renders of the same
    seeds and poses)."""
    w = WORKLOADS["c1_meshrir_plumbing"]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(2)
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=DEV, generator=g) * 0.1
    r = AVRRender(Stub(attn, sig), **w.render)
    gr = GraphedRender(r, ring=3)
    n = 8
    ros = [torch.full((B, 3), 0.1 * k - 0.3) for k in range(n)]  # host poses, one per render
    tx = torch.full((B, 3), 0.3)
    with torch.no_grad():
        torch.manual_seed(42)
        got = [gr.render_ir(ros[k], tx)[1].clone() for k in range(n)]
        torch.manual_seed(42)
        ref = [r.render_ir(ros[k].to(DEV), tx.to(DEV))[1].clone() for k in range(n)]
    torch.cuda.synchronize()
    for k in range(n):
        assert torch.equal(got[k], ref[k]), k
    assert not all(torch.equal(got[0], x) for x in got[1:])  # the jitter did change


def test_graph_host_pose_mixed_devices_and_bad_shapes():
    """Host rays_o with a DEVICE position_tx (or a float64 / strided one)
    is staged by value, not by a host memmove from its pointer, and renders
    as the eager path does; a pose of the wrong size raises instead of
    reading past the tensor."""
    w = WORKLOADS["c1_meshrir_plumbing"]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(5)
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=DEV, generator=g) * 0.1
    r = AVRRender(Stub(attn, sig), **w.render)
    gr = GraphedRender(r, ring=1)
    ro = torch.full((B, 3), 0.25)
    txs = [torch.full((B, 3), -0.4, device=DEV),                  # device tensor beside host rays_o
           torch.full((B, 3), 0.6, dtype=torch.float64),          # another dtype
           torch.full((3, B), 0.2).t()]                           # non-contiguous
    for k, tx in enumerate(txs):
        with torch.no_grad():
            torch.manual_seed(70 + k)
            _, ir_g = gr.render_ir(ro, tx)
            ir_g = ir_g.clone()
            torch.manual_seed(70 + k)
            _, ir_e = r.render_ir(ro.to(DEV), tx.to(DEV, torch.float32))
        torch.cuda.synchronize()
        assert torch.equal(ir_g, ir_e), k
    with pytest.raises(ValueError):
        gr.render_ir(ro, torch.zeros(B + 1, 3, device=DEV))
    with pytest.raises(ValueError):
        gr.render_ir(ro, torch.zeros(B, 2))


@pytest.mark.parametrize("mlp_dtype", [torch.bfloat16, torch.float32])
def test_graph_replay_sees_optimizer_step_avrmodel(mlp_dtype):
    """The package's own network captured (cast/packed-weight caches bypassed
    while capturing): after an in-place Adam step the replay renders with the
    NEW weights, equal to the eager render, and no re-capture happens."""
    from avr_amd.model import AVRModel
    from avr_amd.workloads import MESHRIR, MESHRIR_MODEL

    cfg = dict(MESHRIR, n_azi=16, n_ele=8, n_samples=64)
    torch.manual_seed(0)
    m = AVRModel(dict(MESHRIR_MODEL, signal_output_dim=1022), mlp_dtype=mlp_dtype).to(DEV)
    r = AVRRender(m, **cfg).to(DEV)
    gr = GraphedRender(r)
    g = torch.Generator(device=DEV).manual_seed(3)
    ro = torch.rand(1, 3, device=DEV, generator=g) * 2 - 1
    tx = ro + 0.5  # close source: live windows inside T

    def both(seed):
        with torch.no_grad():
            torch.manual_seed(seed)
            e = r.render_ir(ro, tx)[0].clone()
            torch.manual_seed(seed)
            gg = gr.render_ir(ro, tx)[0].clone()
        torch.cuda.synchronize()
        return e, gg

    e0, g0 = both(5)
    assert e0.abs().max() > 0
    torch.testing.assert_close(g0, e0, rtol=1e-5, atol=1e-6)
    opt = torch.optim.Adam(r.parameters(), lr=1e-2)
    torch.manual_seed(5)
    r(ro, tx).square().sum().backward()
    opt.step()
    e1, g1 = both(5)
    assert (e1 - e0).abs().max() > 1e-4 * e0.abs().max()  # the step changed the render
    torch.testing.assert_close(g1, e1, rtol=1e-5, atol=1e-6)
    assert len(gr._graphs) == 1


def test_graph_replay_propagate_nonfinite():
    """A render with propagate_nonfinite=True captures and replays (the
    poison term uses scalar operands, no host-to-device copy): clean inputs
    replay the eager spectrum bit for bit, a NaN in a masked chunk poisons
    the replayed spectrum as it does the eager one."""
    w = WORKLOADS["c1_meshrir_plumbing"]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(2)
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=DEV, generator=g) * 0.1
    r = AVRRender(Stub(attn, sig), propagate_nonfinite=True, **w.render)
    gr = GraphedRender(r)
    ro = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    tx = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
    with torch.no_grad():
        for k in range(4):
            torch.manual_seed(20 + k)
            out_e, ir_e = r.render_ir(ro, tx)
            torch.manual_seed(20 + k)
            out_g, ir_g = gr.render_ir(ro, tx)
            torch.cuda.synchronize()
            assert torch.isfinite(out_e).all()
            assert torch.equal(out_g, out_e), k
            assert torch.equal(ir_g, ir_e), k
        sig[0, 0, 0] = float("nan")  # replays read the stub's tensor by pointer
        torch.manual_seed(30)
        out_g, ir_g = gr.render_ir(ro, tx)
        torch.cuda.synchronize()
        assert torch.isnan(out_g).all() and torch.isnan(ir_g).all()
