"""Generate golden vectors from the REAL reference renderer (build container only).

Imports `/root/reference/renderer_cpu.py` (it needs only torch + numpy), runs
`AVRRender.forward` with a stub `network_fn` on seeded inputs
(`avr_amd.workloads.make_inputs`) and autograd through it, and writes small
fixtures to `tests/golden/<case>.npz`.  It also runs the repo's own CPU oracle
(`oracle/avr_oracle.py`) on the same inputs and refuses to write a fixture
unless the oracle matches the reference bit for bit, which is what pins the
oracle.

Fixtures hold data only (seeds, shapes, config, expected outputs, checksums);
inputs are regenerated from the seeds by the tests.  Nothing here runs on the
GPU box: `/root/reference` does not exist there.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [case ...]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True

from avr_amd.workloads import WORKLOADS, Workload, MESHRIR, grad_probe, make_inputs  # noqa: E402
from oracle import avr_oracle as orc  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")

W = WORKLOADS
CASES = {
    "c1_s0": (W["c1_meshrir_plumbing"], 0, True),  # every ray-sample masked: all-zero output
    "c1_s1": (W["c1_meshrir_plumbing"], 1, True),
    "c1_s2": (W["c1_meshrir_plumbing"], 2, False),
    "c2_s0": (W["c2_meshrir_1024x256x512"], 0, True),
    "c3_s0": (W["c3_raf_furnished_b4"], 0, True),
    "c4_s0": (W["c4_raf_empty_b4_per_gpu"], 0, True),  # RAF-Empty per-GPU training shard
    # config 5 shapes along S and T (512 samples, T=4094, fp16), fewer rays so
    # the reference fits host RAM
    "c5small_s0": (W["c5_simu_4096x512x2048"].replace(name="c5small", n_azi=4, n_ele=23), 0, True),
    # ragged edge case: asymmetric cube (denormalize offset 5 m), S not a
    # multiple of 32, T = 2 mod 4, single elevation ring, B = 3, low fs so
    # the delays stay inside the signal
    "edge_ragged_s3": (Workload("edge_ragged", dict(MESHRIR, xyz_min=0, xyz_max=10, n_azi=3, n_ele=1,
                                                     n_samples=40, far=3, fs=8000), 250, 3), 3, True),
    # odd T: irfft length becomes 2(F-1) = T-1
    "edge_oddT_s4": (Workload("edge_oddT", dict(MESHRIR, n_azi=5, n_ele=3, n_samples=33), 255, 2,
                              with_dir_tx=True), 4, True),
}

MAX_FULL = 1 << 16  # store arrays in full up to this many elements


def _ref_module():
    sys.path.insert(0, REF)
    import renderer_cpu  # noqa: WPS433  (reference, container only)
    return renderer_cpu


def _sample_idx(n, k, seed):
    rng = np.random.default_rng(777 + seed)
    return np.sort(rng.choice(n, size=min(n, k), replace=False)).astype(np.int64)


def _digest(name, t, seed, store):
    a = t.detach().double().reshape(-1).numpy()
    store[name + "_sum"] = np.array(a.sum())
    store[name + "_sumsq"] = np.array((a * a).sum())
    if a.size <= MAX_FULL:
        store[name] = t.detach().numpy()
    else:
        idx = _sample_idx(a.size, 4096, seed)
        store[name + "_idx"] = idx
        store[name + "_at"] = t.detach().reshape(-1).numpy()[idx]


def run_case(name, w: Workload, seed: int, grads: bool):
    rc = _ref_module()
    inp = make_inputs(w, seed)
    rays_o = torch.from_numpy(inp["rays_o"])
    tx = torch.from_numpy(inp["position_tx"])
    dtx = None if inp["direction_tx"] is None else torch.from_numpy(inp["direction_tx"])
    attn = torch.from_numpy(inp["attn"]).requires_grad_(grads)
    signal = torch.from_numpy(inp["signal"]).requires_grad_(grads)

    # --- reference forward (+ backward) ---
    stub = orc.StubNetwork(attn, signal)
    ref = rc.AVRRender(stub, **w.render)
    torch.manual_seed(seed)
    t0 = time.time()
    out_ref = ref(rays_o, tx, dtx) if dtx is not None else ref(rays_o, tx)
    t_fwd = time.time() - t0
    seen = stub.seen
    store = {}
    if grads:
        g = torch.from_numpy(grad_probe(w, seed))
        (out_ref * g).sum().backward()
        store["grad_probe_seed"] = np.array(seed)
        _digest("grad_attn", attn.grad, seed, store)
        _digest("grad_signal", signal.grad, seed, store)
        store["grad_signal_dot_signal"] = np.array(
            (signal.grad.double() * signal.detach().double()).sum().item())

    # --- reference stages called directly ---
    torch.manual_seed(seed)
    dirs_ref, _, _ = rc.ray_directions(w.render["n_azi"], w.render["n_ele"])
    S = w.n_samples
    # weights through the reference's own acoustic_render with a one-hot signal
    d_vals = torch.linspace(0.0, 1.0, S) * (w.render["far"] - w.render["near"]) + w.render["near"]
    a3 = attn.detach().float().view(w.batch, -1, S)
    eye = torch.eye(S).expand(w.batch, a3.size(1), S, S)
    w_ref = rc.acoustic_render(a3, eye, d_vals)

    # --- oracle, same seed: must be bit-identical ---
    rec = {}
    torch.manual_seed(seed)
    stub2 = orc.StubNetwork(attn.detach(), signal.detach())
    cfg = orc.RenderConfig.from_kwargs(**w.render)
    out_orc = orc.render_spectrum(cfg, stub2, rays_o, tx, dtx, record=rec)
    checks = {
        "out": torch.equal(out_orc, out_ref.detach()),
        "dirs": torch.equal(rec["dirs"], dirs_ref),
        "weights": torch.equal(rec["weights"], w_ref),
        "pts": torch.equal(rec["pts"], seen[0]),
        "view": torch.equal(rec["view"], seen[1]),
        "tx": torch.equal(rec["tx"], seen[2]),
    }
    if dtx is not None:
        checks["dir_tx"] = torch.equal(rec["dir_tx"], seen[3])
    bad = [k for k, v in checks.items() if not v]
    if bad:
        diff = (out_orc - out_ref.detach()).abs().max().item()
        raise SystemExit(f"{name}: oracle differs from reference in {bad} (max |d out| = {diff})")

    ir_ref = orc.spectrum_to_ir(out_ref.detach())
    meta = dict(case=name, workload=w.name, render=w.render, T=w.T, batch=w.batch,
                with_dir_tx=w.with_dir_tx, signal_dtype=w.signal_dtype,
                attn_dtype=w.attn_dtype, seed=seed, grads=grads,
                ref_forward_seconds=round(t_fwd, 4), torch=torch.__version__)
    store.update(
        meta=np.array(json.dumps(meta)),
        u_azi=rec["u_azi"].numpy(),
        dirs=dirs_ref.numpy(),
        d_vals=d_vals.numpy(),
        shift=rec["shift"].numpy(),
        out=out_ref.detach().numpy(),
        ir=ir_ref.numpy(),
    )
    _digest("weights", w_ref, seed, store)
    # integer delays are stored in full at every size: they are compared
    # bit for bit (a single flipped delay moves a whole masked window)
    dl = rec["delay"].detach()
    assert float(dl.max()) < 32768
    store["delay"] = dl.numpy().astype(np.int16)
    store["delay_sum"] = np.array(float(dl.double().sum()))
    for k, t in zip(("pts", "view", "tx", "dir_tx"), seen):
        if t is not None:
            _digest("net_" + k, t, seed, store)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **store)
    print(f"{name}: ok ({os.path.getsize(path) / 1024:.1f} KiB, ref fwd {t_fwd:.2f}s)", flush=True)


def main(argv):
    os.makedirs(OUT, exist_ok=True)
    names = argv or list(CASES)
    for n in names:
        w, seed, grads = CASES[n]
        run_case(n, w, seed, grads)


if __name__ == "__main__":
    main(sys.argv[1:])
