"""Reentrancy: nn.DataParallel (avr_runner.py:63) calls forward from one host
thread per device, concurrently.  Here two host threads share ONE AVRRender
(and so its parameter cache, the per-device tables and the library's launch
state), each issuing renders on its own HIP stream; every result must be
bitwise equal to the same render issued serially."""
import threading

import pytest
import torch

from avr_amd import AVRRender
from avr_amd.model import AVRModel_complex
from avr_amd.workloads import RAF, RAF_MODEL, WORKLOADS

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class Stub(torch.nn.Module):
    def __init__(self, attn, signal):
        super().__init__()
        self.attn, self.signal = attn, signal

    def forward(self, pts, view, tx, dir_tx=None):
        return self.attn, self.signal


def _poses(n, seed, dir_tx=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    out = []
    for _ in range(n):
        ro = torch.rand(1, 3, device=DEV, generator=g) * 4 - 2
        tx = torch.rand(1, 3, device=DEV, generator=g) * 4 - 2
        d = torch.nn.functional.normalize(torch.randn(1, 3, device=DEV, generator=g), dim=-1) if dir_tx else None
        out.append((ro, tx, d))
    return out


def _run_threads(render, poses_per_thread):
    """Each thread renders its pose list on its own stream; the azimuth jitter
    (CPU generator, not thread-safe by design in the reference either) is
    fixed per pose with u_azi so results are comparable."""
    results = [[None] * len(p) for p in poses_per_thread]
    errors = []
    barrier = threading.Barrier(len(poses_per_thread))

    def body(k):
        try:
            s = torch.cuda.Stream(DEV)
            torch.cuda.set_device(DEV)
            barrier.wait()
            with torch.cuda.stream(s), torch.no_grad():
                for i, args in enumerate(poses_per_thread[k]):
                    results[k][i] = render(*args)
            s.synchronize()
        except Exception as e:  # surfaced in the main thread
            errors.append(e)

    ts = [threading.Thread(target=body, args=(k,)) for k in range(len(poses_per_thread))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors
    return results


def _jitter(n_azi, seed):
    return torch.rand(n_azi, generator=torch.Generator().manual_seed(seed))


def test_two_threads_share_one_renderer_stub_network():
    w = WORKLOADS["c2_meshrir_1024x256x512"]
    R, S, T = w.n_rays, w.n_samples, w.T
    g = torch.Generator(device=DEV).manual_seed(0)
    attn = torch.rand(1, R * S, 1, device=DEV, generator=g) * 2
    sig = torch.randn(1, R * S, T, device=DEV, generator=g) * 0.1
    r = AVRRender(Stub(attn, sig), **w.render)

    def render(ro, tx, _d, u):
        pts, view, txn, dtx, geom = r.sample(ro, tx, None, u_azi=u)
        a, s = r.network_fn(pts, view, txn)
        return r.render_from_network_output(a, s, geom)

    poses = [[(*p, _jitter(w.render["n_azi"], 10 * k + i)) for i, p in enumerate(_poses(6, k))]
             for k in range(2)]
    par = _run_threads(render, poses)
    torch.cuda.synchronize()
    with torch.no_grad():
        for k in range(2):
            for i, args in enumerate(poses[k]):
                assert torch.equal(par[k][i], render(*args)), (k, i)


def test_two_threads_share_one_renderer_fused_head_model():
    cfg = dict(RAF, n_azi=12, n_ele=6, n_samples=32)
    torch.manual_seed(0)
    m = AVRModel_complex(dict(RAF_MODEL, signal_output_dim=800)).to(DEV)
    r = AVRRender(m, **cfg).to(DEV)

    def render(ro, tx, d, u):
        pts, view, txn, dtx, geom = r.sample(ro, tx, d, u_azi=u)
        attn, h, weight, dtype = m.forward_fused(pts, view, txn, dtx,
                                                 ray_layout=(1, geom["n_rays"], cfg["n_samples"]))
        return r.render_from_hidden(attn, h, weight, dtype, geom)

    poses = [[(*p, _jitter(cfg["n_azi"], 10 * k + i)) for i, p in enumerate(_poses(4, 5 + k, True))]
             for k in range(2)]
    par = _run_threads(render, poses)
    torch.cuda.synchronize()
    with torch.no_grad():
        for k in range(2):
            for i, args in enumerate(poses[k]):
                assert torch.equal(par[k][i], render(*args)), (k, i)
