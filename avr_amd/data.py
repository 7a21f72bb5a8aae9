"""Dataset and result formats around the render path.

* `WaveLoader` — the reference's `datasets_loader.WaveLoader`
  (datasets_loader.py:10-220): same constructor, same four dataset layouts,
  same items (complex64 spectrum of the IR window, positions, RAF source
  orientation, channel index).
    MeshRIR:  <base>/{train,test}/*_<idx>.npy  [C, samples] at 48 kHz,
              <base>/pos_mic.npy [N, 3], <base>/pos_src.npy [1, 3]
    Simu:     <base>/*.npz with ir, position_rx, position_tx (90/10 split)
    Real_env: <base>/train_test_split.pkl {"train": [...], "test": [...]}
              of .npz files with ir, position_rx, position_tx[, ch_idx]
    RAF:      <base>/{train,test}/<id>/rir.wav, rx_pos.txt, tx_pos.txt
  `librosa.load(sr=None, mono=True)` (datasets_loader.py:165) is replaced by
  `read_wav` (RIFF PCM 8/16/24/32-bit and IEEE float, channels averaged),
  because librosa is not available; values follow libsndfile's scaling.
  The split pickle is read with an unpickler that only builds plain
  containers (no class lookups), so a split file cannot run code.
* `write_val_dump` / `read_val_dump` — the `val_iter%06d.npz` files of
  avr_runner.py:278-302 (ori_sig / pred_sig complex [N, F], positions,
  optional ch_idx, fs), which the DoA and plotting scripts read.

Host-side I/O only: the spectra go to the GPU as the reference's loop sends
them (`ori_sig.cuda()`, avr_runner.py:179).
"""
from __future__ import annotations

import glob
import io
import math
import os
import pickle
import struct

import numpy as np
import torch
from torch.utils.data import Dataset


# ------------------------------------------------------------------ WAV
def read_wav(path):
    """(samples float32 mono, sample_rate) of a RIFF/WAVE file.

    PCM is scaled as libsndfile does (int16 / 2^15, 24-bit and 32-bit as
    int32 / 2^31, 8-bit unsigned (x - 128) / 2^7); IEEE float is returned
    as stored; channels are averaged (librosa.to_mono)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos = 12
    fmt = None
    payload = None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, rate, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: subformat GUID
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, rate, bits)
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, rate, bits = fmt
    width = bits // 8
    payload = payload[:len(payload) - len(payload) % (width * ch)]
    if tag == 1:  # PCM
        if bits == 8:
            x = (np.frombuffer(payload, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(payload, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(payload, np.uint8).reshape(-1, 3).astype(np.int32)
            v = (b[:, 0] << 8) | (b[:, 1] << 16) | (b[:, 2] << 24)
            x = (v.astype(np.float64) / 2147483648.0).astype(np.float32)
        elif bits == 32:
            x = (np.frombuffer(payload, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
        else:
            raise ValueError(f"{path}: unsupported PCM width {bits}")
    elif tag == 3:  # IEEE float
        x = np.frombuffer(payload, "<f4" if bits == 32 else "<f8").astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported WAVE format tag {tag}")
    x = x.reshape(-1, ch)
    mono = x[:, 0] if ch == 1 else np.mean(x, axis=1, dtype=np.float32)
    return np.ascontiguousarray(mono, dtype=np.float32), rate


def write_wav(path, samples, rate, bits=16):
    """Mono PCM / float WAV writer (tests and tools)."""
    x = np.asarray(samples)
    if bits == 16:
        raw = np.clip(np.round(x * 32768.0), -32768, 32767).astype("<i2").tobytes()
        tag = 1
    elif bits == 32:
        raw = x.astype("<f4").tobytes()
        tag = 3
    else:
        raise ValueError("bits must be 16 (PCM) or 32 (float)")
    fmt = struct.pack("<HHIIHH", tag, 1, rate, rate * bits // 8, bits // 8, bits)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(raw)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt)) + fmt)
        f.write(b"data" + struct.pack("<I", len(raw)) + raw)


class _PlainUnpickler(pickle.Unpickler):
    """Builds dicts / lists / tuples / strings / numbers only."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"split file references {module}.{name}; only plain "
                                     "containers are accepted")


def load_split(path):
    with open(path, "rb") as f:
        return _PlainUnpickler(io.BytesIO(f.read())).load()


def quaternion_to_direction_vector(q):
    """datasets_loader.py:223-245: forward vector of an [x, y, z, w]
    quaternion, projected to the floor plane and negated, with the reference's
    axis order."""
    x, y, z, w = q
    fwd_x = 2 * (x * z + w * y)
    fwd_z = 1 - 2 * (x * x + y * y)
    norm = math.sqrt(fwd_x ** 2 + 0 ** 2 + fwd_z ** 2)
    return np.array([-fwd_x / norm, -fwd_z / norm, 0])


# ------------------------------------------------------------- datasets
class WaveLoader(Dataset):
    """datasets_loader.WaveLoader: spectra + poses of one split."""

    def __init__(self, base_folder, dataset_type='MeshRIR', eval=False, seq_len=2048, fs=16000):
        self.wave_chunks = []
        self.positions_rx = []
        self.positions_tx = []
        self.rotations_tx = []
        self.ch_idx_list = []
        self.wave_max = float('-inf')
        self.wave_min = float('inf')
        self.position_max = np.array([float('-inf')] * 3)
        self.position_min = np.array([float('inf')] * 3)
        self.dataset_type = dataset_type
        self.eval = eval
        loaders = {'MeshRIR': self.load_mesh_rir, 'RAF': self.load_raf,
                   'Simu': self.load_simu, 'Real_env': self.load_real_env}
        if dataset_type not in loaders:
            raise ValueError("Unsupported dataset type")
        loaders[dataset_type](base_folder, eval, seq_len, fs)
        self.wave_chunks = torch.tensor(np.array(self.wave_chunks), dtype=torch.complex64)
        self.positions_rx = torch.tensor(np.array(self.positions_rx), dtype=torch.float32)
        self.positions_tx = torch.tensor(np.array(self.positions_tx), dtype=torch.float32)
        if self.rotations_tx:
            self.rotations_tx = torch.tensor(np.array(self.rotations_tx), dtype=torch.float32)

    def _add(self, audio, rx, tx):
        self.wave_max = max(self.wave_max, audio.max())
        self.wave_min = min(self.wave_min, audio.min())
        self.position_max = np.maximum(self.position_max, rx)
        self.position_min = np.minimum(self.position_min, rx)
        self.wave_chunks.append(np.fft.rfft(audio))
        self.positions_rx.append(rx)
        self.positions_tx.append(tx)

    def load_mesh_rir(self, base_folder, eval, seq_len, fs=24000):
        """datasets_loader.py:61-91: 48 kHz IRs decimated to fs, window from
        sample 9100/decimation."""
        down = 48000 // fs
        self.default_st_idx = int(9100 / down)
        folder = os.path.join(base_folder, 'test' if eval else 'train')
        names = sorted(f for f in os.listdir(folder) if f.endswith('.npy'))
        rx_pos = np.load(os.path.join(base_folder, 'pos_mic.npy'))
        tx_pos = np.load(os.path.join(base_folder, 'pos_src.npy'))[0]
        for name in names:
            audio = np.load(os.path.join(folder, name))[0, ::down]
            audio = audio[self.default_st_idx:self.default_st_idx + seq_len]
            idx = int(name.split('_')[1].split('.')[0])
            self._add(audio, rx_pos[idx], tx_pos)

    def load_simu(self, base_folder, eval, seq_len, fs):
        """datasets_loader.py:93-116: sorted .npz files, first 90% train."""
        names = sorted(f for f in os.listdir(base_folder) if f.endswith('.npz'))
        cut = int(0.9 * len(names))
        names = names[cut:] if eval else names[:cut]
        for name in names:
            meta = np.load(os.path.join(base_folder, name))
            self._add(meta['ir'][:seq_len], meta['position_rx'], meta['position_tx'])

    def load_real_env(self, base_folder, eval, seq_len, fs):
        """datasets_loader.py:118-149: predefined split, optional ch_idx."""
        split = load_split(os.path.join(base_folder, "train_test_split.pkl"))
        for path in (split["test"] if eval else split["train"]):
            if not os.path.isabs(path):
                path = os.path.join(base_folder, path)
            meta = np.load(path)
            self._add(meta['ir'][:seq_len], meta['position_rx'], meta['position_tx'])
            if "ch_idx" in meta:
                self.ch_idx_list.append(meta["ch_idx"].item())

    def load_raf(self, base_folder, eval, seq_len, fs):
        """datasets_loader.py:151-177: rir.wav decimated from 48 kHz,
        rx_pos.txt / tx_pos.txt (quaternion then position), y/z swapped."""
        folders = sorted(glob.glob(f"{base_folder}/{'test' if eval else 'train'}/*"))
        step = int(48000 / fs)
        for folder in folders:
            audio, _ = read_wav(os.path.join(folder, "rir.wav"))
            audio = audio[:seq_len * step:step]
            rx = self.load_position(os.path.join(folder, "rx_pos.txt"))
            tx, rot = self.load_tx_info(os.path.join(folder, "tx_pos.txt"))
            self._add(audio, rx, tx)
            self.rotations_tx.append(rot)

    @staticmethod
    def _numbers(path):
        vals = []
        with open(path) as f:
            for line in f:
                vals.extend(float(v) for v in line.split(','))
        return np.array(vals)

    def load_position(self, file_path):
        return self._numbers(file_path)[[0, 2, 1]]

    def load_tx_info(self, file_path):
        info = self._numbers(file_path)
        return np.array(info[4:])[[0, 2, 1]], quaternion_to_direction_vector(info[:4])

    def __len__(self):
        return len(self.wave_chunks)

    def __getitem__(self, idx):
        """datasets_loader.py:206-220 (RAF training poses jittered by 0.1 m)."""
        wave = self.wave_chunks[idx]
        rx = self.positions_rx[idx]
        tx = self.positions_tx[idx]
        ch_idx = self.ch_idx_list[idx] if len(self.ch_idx_list) > 0 else -1
        if not self.eval and self.dataset_type == 'RAF':
            rx = rx + torch.randn_like(rx) * 0.1
            tx = tx + torch.randn_like(tx) * 0.1
        if self.dataset_type == 'RAF':
            return wave, rx, tx, self.rotations_tx[idx], ch_idx
        return wave, rx, tx, ch_idx


# ------------------------------------------------------------ val dumps
def write_val_dump(path, ori_sig, pred_sig, position_rx, position_tx, fs, ch_idx=None):
    """avr_runner.py:278-302: val_iter%06d.npz (lists are concatenated on axis 0)."""
    cat = lambda v: np.concatenate([np.asarray(a) for a in v], axis=0) if isinstance(v, (list, tuple)) \
        else np.asarray(v)
    arrays = dict(ori_sig=cat(ori_sig), pred_sig=cat(pred_sig), position_rx=cat(position_rx),
                  position_tx=cat(position_tx))
    if ch_idx is not None and (not isinstance(ch_idx, (list, tuple)) or len(ch_idx) > 0):
        arrays["ch_idx"] = cat(ch_idx)
    np.savez_compressed(path, fs=fs, **arrays)
    return path


def read_val_dump(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def val_dump_name(iteration):
    return f"val_iter{iteration:06d}.npz"
