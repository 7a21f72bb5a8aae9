"""Synthetic datasets in the reference's four on-disk layouts
(datasets_loader.py:61-177), built deterministically from a seed.  Shared by
tests/test_data_formats.py and tools/gen_data_golden.py, which runs the
reference's own WaveLoader on them and stores its outputs in
tests/golden/data/."""
import os
import pickle

import numpy as np

from avr_amd.data import write_wav

# name -> (layout, loader kwargs)
CASES = {
    "meshrir": ("MeshRIR", dict(seq_len=1022, fs=24000)),
    "simu": ("Simu", dict(seq_len=800, fs=16000)),
    "real_env": ("Real_env", dict(seq_len=640, fs=16000)),
    "raf": ("RAF", dict(seq_len=400, fs=16000)),
}


def build(name, root, seed=0):
    """Write dataset `name` under root/<name>; returns its base folder."""
    rng = np.random.default_rng(seed)
    base = os.path.join(root, name)
    os.makedirs(base, exist_ok=True)
    if name == "meshrir":
        for split in ("train", "test"):
            os.makedirs(os.path.join(base, split), exist_ok=True)
        np.save(os.path.join(base, "pos_mic.npy"), rng.standard_normal((12, 3)))
        np.save(os.path.join(base, "pos_src.npy"), rng.standard_normal((1, 3)))
        for split, ids in (("train", (7, 2, 11, 5)), ("test", (3, 9))):
            for i in ids:
                np.save(os.path.join(base, split, f"ir_{i}.npy"), rng.standard_normal((1, 12000)) * 0.1)
    elif name == "simu":
        for i in range(11):  # 90/10 split of sorted names: 9 train, 2 test
            np.savez(os.path.join(base, f"sample_{i:03d}.npz"),
                     ir=(rng.standard_normal(1000) * 0.05).astype(np.float32),
                     position_rx=rng.uniform(-3, 3, 3), position_tx=rng.uniform(-3, 3, 3))
    elif name == "real_env":
        files = []
        for i in range(7):
            rel = f"env_{i}.npz"
            np.savez(os.path.join(base, rel), ir=rng.standard_normal(900) * 0.05,
                     position_rx=rng.uniform(-3, 3, 3), position_tx=rng.uniform(-3, 3, 3),
                     ch_idx=np.array(int(rng.integers(0, 8))))
            files.append(rel)
        with open(os.path.join(base, "train_test_split.pkl"), "wb") as f:
            pickle.dump({"train": files[:5], "test": files[5:]}, f)
    elif name == "raf":
        for split, n in (("train", 4), ("test", 2)):
            for i in range(n):
                d = os.path.join(base, split, f"{i:05d}")
                os.makedirs(d, exist_ok=True)
                write_wav(os.path.join(d, "rir.wav"), (rng.standard_normal(1500) * 0.1).astype(np.float32),
                          48000, bits=16)
                rx = rng.uniform(-4, 4, 3)
                q = rng.standard_normal(4)
                q /= np.linalg.norm(q)
                tx = rng.uniform(-4, 4, 3)
                with open(os.path.join(d, "rx_pos.txt"), "w") as f:
                    f.write(",".join(f"{v:.6f}" for v in rx) + "\n")
                with open(os.path.join(d, "tx_pos.txt"), "w") as f:
                    f.write(",".join(f"{v:.6f}" for v in q) + "\n")
                    f.write(",".join(f"{v:.6f}" for v in tx) + "\n")
    else:
        raise KeyError(name)
    return base


def summarize(ds):
    """The loader state the fixtures pin (numpy arrays)."""
    out = {
        "wave_chunks": ds.wave_chunks.numpy(),
        "positions_rx": ds.positions_rx.numpy(),
        "positions_tx": ds.positions_tx.numpy(),
        "wave_max_min": np.array([ds.wave_max, ds.wave_min], np.float64),
        "position_max": np.asarray(ds.position_max, np.float64),
        "position_min": np.asarray(ds.position_min, np.float64),
        "ch_idx": np.array(ds.ch_idx_list if ds.ch_idx_list else [-1] * len(ds), np.int64),
    }
    if ds.dataset_type == "RAF":
        out["rotations_tx"] = ds.rotations_tx.numpy()
    return out
