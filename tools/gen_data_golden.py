"""Golden outputs of the REAL reference `datasets_loader.WaveLoader` on the
synthetic datasets of tests/data_cases.py, all four layouts, train and eval
splits (build container only).

librosa (used only by the RAF layout, `librosa.load(rir_path, sr=None,
mono=True)`, datasets_loader.py:165) is not installed.  Its import is
satisfied by a placeholder whose `load` decodes the fixture's 16-bit PCM mono
WAV with scipy.io.wavfile as int16 / 32768 in float32, which is what librosa
returns for such a file (it reads through soundfile, PCM_16 -> float32 scaled
by 1/32768).  Everything else -- file discovery and sorting, splits,
decimation, windows, rfft, axis swaps, the quaternion rule, min/max
tracking, the split pickle -- runs the reference's own code.

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_data_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "data")

from data_cases import CASES, build, summarize  # noqa: E402


def _reference_loader():
    from scipy.io import wavfile

    def load(path, sr=None, mono=True):
        assert sr is None and mono
        rate, x = wavfile.read(path)
        assert x.dtype == np.int16 and x.ndim == 1, "fixtures are 16-bit PCM mono"
        return x.astype(np.float32) / np.float32(32768.0), rate

    lib = types.ModuleType("librosa")
    lib.load = load
    sys.modules["librosa"] = lib
    sys.path.insert(0, REF)
    import datasets_loader  # noqa: E402  (the reference's file)

    return datasets_loader.WaveLoader


def main():
    WaveLoader = _reference_loader()
    os.makedirs(OUT, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        for name, (layout, kw) in CASES.items():
            base = build(name, tmp)
            for ev in (False, True):
                ds = WaveLoader(base, layout, eval=ev, **kw)
                z = summarize(ds)
                import torch

                torch.manual_seed(123)  # RAF training items are jittered (datasets_loader.py:213-215)
                items = [ds[i] for i in range(len(ds))]
                for k, it in enumerate(items):
                    z[f"item{k}_wave"] = it[0].numpy()
                    z[f"item{k}_rx"] = it[1].numpy()
                    z[f"item{k}_tx"] = it[2].numpy()
                z["meta"] = json.dumps(dict(name=name, layout=layout, eval=ev, kw=kw, n=len(ds),
                                            items=len(items), source="datasets_loader.py (reference)"))
                tag = f"{name}_{'eval' if ev else 'train'}"
                np.savez_compressed(os.path.join(OUT, f"{tag}.npz"), **z)
                print(tag, len(ds), {k: v.shape for k, v in z.items() if k != "meta" and not k.startswith("item")})


if __name__ == "__main__":
    main()
