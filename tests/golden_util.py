"""Load tests/golden/*.npz fixtures (written by tools/gen_golden.py from the
real reference) and regenerate their inputs from the stored seeds."""
from __future__ import annotations

import glob
import json
import os

import numpy as np

from avr_amd.workloads import Workload, grad_probe, make_inputs

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


class Case:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.meta = json.loads(str(self.z["meta"]))
        m = self.meta
        self.workload = Workload(m["workload"], dict(m["render"]), m["T"], m["batch"],
                                 with_dir_tx=m["with_dir_tx"], signal_dtype=m["signal_dtype"],
                                 attn_dtype=m["attn_dtype"])
        self.seed = m["seed"]
        self.grads = m["grads"]

    def inputs(self):
        return make_inputs(self.workload, self.seed)

    def grad_probe(self):
        return grad_probe(self.workload, self.seed)

    def has(self, key):
        return key in self.z

    def __getitem__(self, key):
        return self.z[key]


def digest_check(case, name, actual, rtol=0.0, atol=0.0):
    """Compare `actual` (numpy) to a stored digest (full array or samples)."""
    a = np.asarray(actual)
    if case.has(name):
        np.testing.assert_allclose(a, case[name], rtol=rtol, atol=atol)
    else:
        flat = a.reshape(-1)
        np.testing.assert_allclose(flat[case[name + "_idx"]], case[name + "_at"], rtol=rtol, atol=atol)
    s = float(a.astype(np.float64).sum())
    ss = float((a.astype(np.float64) ** 2).sum())
    return s, ss


def rel_l2(a, b):
    """||a-b|| / ||b|| (absolute when b is all zero: fully masked cases)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    d = np.linalg.norm(a - b)
    return float(d / nb) if nb > 0 else float(d)


def rel_max(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    mb = np.abs(b).max() if b.size else 0.0
    d = np.abs(a - b).max() if b.size else 0.0
    return float(d / mb) if mb > 0 else float(d)
