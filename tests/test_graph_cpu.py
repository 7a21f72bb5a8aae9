"""Host-side facts the HIP-graph replay (avr_amd.graph) relies on: one CPU
draw of n_azi + n_ele uniforms equals the reference's two draws
(renderer.py:149,153) value for value and leaves the generator in the same
state, for every workload's sphere."""
import pytest
import torch

from avr_amd.workloads import WORKLOADS


@pytest.mark.parametrize("name", sorted(WORKLOADS))
def test_one_draw_equals_two(name):
    r = WORKLOADS[name].render
    a, b = int(r["n_azi"]), int(r["n_ele"])
    torch.manual_seed(11)
    u, e, nxt = torch.rand(a), torch.rand(b), torch.rand(7)
    torch.manual_seed(11)
    buf = torch.empty(a + b)
    torch.rand(a + b, out=buf)
    assert torch.equal(buf[:a], u) and torch.equal(buf[a:], e)
    assert torch.equal(torch.rand(7), nxt)
