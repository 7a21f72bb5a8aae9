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
    def __init__(self, a, s):
        super().__init__()
        self.a, self.s = a, s

    def forward(self, *args, **kw):
        return self.a, self.s


@pytest.mark.parametrize("name", ["c2_meshrir_1024x256x512", "c3_raf_furnished_b4"])
def test_graph_replay_equals_eager(name):
    w = WORKLOADS[name]
    B, R, S, T = w.batch, w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(1)
    attn = torch.rand(B, R * S, 1, device=DEV, generator=g) * 2
    sig = torch.randn(B, R * S, T, device=DEV, generator=g) * 0.1
    r = AVRRender(Stub(attn, sig), **w.render)
    gr = GraphedRender(r)
    for k in range(3):  # capture, then replays with new poses and jitter
        ro = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
        tx = torch.rand(B, 3, device=DEV, generator=g) * 4 - 2
        dtx = (torch.nn.functional.normalize(torch.randn(B, 3, device=DEV, generator=g), dim=-1)
               if w.with_dir_tx else None)
        with torch.no_grad():
            torch.manual_seed(10 + k)
            out_e, ir_e = r.render_ir(ro, tx, dtx)
            torch.manual_seed(10 + k)
            out_g, ir_g = gr.render_ir(ro, tx, dtx)
            torch.cuda.synchronize()
        assert torch.equal(out_g, out_e), k
        assert torch.equal(ir_g, ir_e), k
    assert len(gr._graphs) == 1
