"""CPU: dataset loaders and result formats (avr_amd/data.py, SURVEY.md §8f
ranks 3-4) on synthetic files laid out as the reference expects them
(datasets_loader.py:61-177, avr_runner.py:278-302).

datasets_loader.py imports librosa (absent), so these tests pin the loaders
to the reference's documented slicing / axis rules, restated in the checks
below, and the WAV reader to scipy's (parity with librosa unpinned)."""
import os
import pickle

import numpy as np
import pytest
import torch
from scipy.io import wavfile

from avr_amd import data


def test_read_wav_matches_scipy_pcm16_and_float(tmp_path):
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(1000) * 0.2).astype(np.float32)
    p16 = tmp_path / "a.wav"
    data.write_wav(str(p16), x, 48000, bits=16)
    rate, raw = wavfile.read(str(p16))
    got, r = data.read_wav(str(p16))
    assert r == rate == 48000
    np.testing.assert_array_equal(got, raw.astype(np.float32) / 32768.0)
    pf = tmp_path / "b.wav"
    data.write_wav(str(pf), x, 16000, bits=32)
    got, r = data.read_wav(str(pf))
    np.testing.assert_array_equal(got, x)


def test_read_wav_stereo_and_24bit(tmp_path):
    rng = np.random.default_rng(1)
    st = (rng.standard_normal((500, 2)) * 3000).astype(np.int16)
    p = tmp_path / "s.wav"
    wavfile.write(str(p), 48000, st)
    got, _ = data.read_wav(str(p))
    np.testing.assert_allclose(got, (st.astype(np.float32) / 32768.0).mean(axis=1), rtol=0, atol=1e-7)
    # 24-bit PCM: build the bytes by hand
    v = rng.integers(-2 ** 23, 2 ** 23, 300)
    b = np.stack([(v >> s) & 0xFF for s in (0, 8, 16)], axis=1).astype(np.uint8).tobytes()
    import struct
    fmt = struct.pack("<HHIIHH", 1, 1, 48000, 48000 * 3, 3, 24)
    p24 = tmp_path / "c.wav"
    with open(p24, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + 8 + 16 + 8 + len(b)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(b)) + b)
    got, _ = data.read_wav(str(p24))
    np.testing.assert_allclose(got, v / 2 ** 23, rtol=0, atol=1e-7)


def test_mesh_rir_loader(tmp_path):
    rng = np.random.default_rng(2)
    base = tmp_path / "mesh"
    (base / "train").mkdir(parents=True)
    (base / "test").mkdir()
    pos_mic = rng.standard_normal((5, 3))
    np.save(base / "pos_mic.npy", pos_mic)
    np.save(base / "pos_src.npy", rng.standard_normal((1, 3)))
    irs = {}
    for i in (3, 1):
        irs[i] = rng.standard_normal((1, 32768))
        np.save(base / "train" / f"ir_{i}.npy", irs[i])
    ds = data.WaveLoader(str(base), "MeshRIR", eval=False, seq_len=1022, fs=24000)
    assert len(ds) == 2
    # sorted file order: ir_1 then ir_3; 48k -> 24k decimation, window from 9100 // 2
    for j, i in enumerate((1, 3)):
        audio = irs[i][0, ::2][4550:4550 + 1022]
        np.testing.assert_allclose(ds.wave_chunks[j].numpy(), np.fft.rfft(audio).astype(np.complex64))
        np.testing.assert_allclose(ds.positions_rx[j].numpy(), pos_mic[i].astype(np.float32))
    wave, rx, tx, ch = ds[0]
    assert wave.dtype == torch.complex64 and wave.shape == (512,) and ch == -1


def test_simu_and_real_env_loaders(tmp_path):
    rng = np.random.default_rng(3)
    base = tmp_path / "simu"
    base.mkdir()
    for i in range(10):
        np.savez(base / f"s{i:02d}.npz", ir=rng.standard_normal(5000),
                 position_rx=rng.standard_normal(3), position_tx=rng.standard_normal(3))
    tr = data.WaveLoader(str(base), "Simu", eval=False, seq_len=4094)
    te = data.WaveLoader(str(base), "Simu", eval=True, seq_len=4094)
    assert len(tr) == 9 and len(te) == 1 and tr.wave_chunks.shape == (9, 2048)

    real = tmp_path / "real"
    real.mkdir()
    files = []
    for i in range(4):
        name = f"r{i}.npz"
        np.savez(real / name, ir=rng.standard_normal(3000), position_rx=rng.standard_normal(3),
                 position_tx=rng.standard_normal(3), ch_idx=np.array(i % 8))
        files.append(name)
    with open(real / "train_test_split.pkl", "wb") as f:
        pickle.dump({"train": files[:3], "test": files[3:]}, f)
    ds = data.WaveLoader(str(real), "Real_env", eval=False, seq_len=1600)
    assert len(ds) == 3 and ds[2][3] == 2


def test_split_loader_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    p = tmp_path / "train_test_split.pkl"
    with open(p, "wb") as f:
        pickle.dump({"train": [Evil()], "test": []}, f)
    with pytest.raises(pickle.UnpicklingError):
        data.load_split(str(p))


def test_raf_loader(tmp_path):
    rng = np.random.default_rng(4)
    base = tmp_path / "raf"
    for split in ("train", "test"):
        for k in range(2):
            d = base / split / f"{k:05d}"
            d.mkdir(parents=True)
            data.write_wav(str(d / "rir.wav"), rng.standard_normal(6000) * 0.1, 48000)
            (d / "rx_pos.txt").write_text("1.0,2.0,3.0\n")
            q = rng.standard_normal(4)
            q /= np.linalg.norm(q)
            (d / "tx_pos.txt").write_text(",".join(map(str, q)) + "\n4.0,5.0,6.0\n")
    ds = data.WaveLoader(str(base), "RAF", eval=True, seq_len=1600, fs=16000)
    assert len(ds) == 2
    wave, rx, tx, rot, ch = ds[0]
    np.testing.assert_allclose(rx.numpy(), [1.0, 3.0, 2.0])  # y/z swapped
    np.testing.assert_allclose(tx.numpy(), [4.0, 6.0, 5.0])
    assert wave.shape == (801,) and rot.shape == (3,) and float(rot[2]) == 0.0
    assert abs(float(rot[:2].norm()) - 1.0) < 1e-6
    audio, _ = data.read_wav(str(base / "test" / "00000" / "rir.wav"))
    np.testing.assert_allclose(wave.numpy(), np.fft.rfft(audio[:1600 * 3:3]).astype(np.complex64),
                               rtol=1e-5, atol=1e-6)


def test_val_dump_round_trip(tmp_path):
    rng = np.random.default_rng(5)
    ori = [rng.standard_normal((2, 801)) + 1j * rng.standard_normal((2, 801)) for _ in range(3)]
    pred = [o * 0.9 for o in ori]
    rx = [rng.standard_normal((2, 3)).astype(np.float32) for _ in range(3)]
    tx = [rng.standard_normal((2, 3)).astype(np.float32) for _ in range(3)]
    p = tmp_path / data.val_dump_name(20000)
    assert p.name == "val_iter020000.npz"
    data.write_val_dump(str(p), [o.astype(np.complex64) for o in ori],
                        [o.astype(np.complex64) for o in pred], rx, tx, fs=16000)
    z = data.read_val_dump(str(p))
    assert set(z) == {"ori_sig", "pred_sig", "position_rx", "position_tx", "fs"}
    assert z["ori_sig"].shape == (6, 801) and z["ori_sig"].dtype == np.complex64
    assert int(z["fs"]) == 16000
    data.write_val_dump(str(p), ori, pred, rx, tx, fs=16000, ch_idx=[np.array([0, 1])] * 3)
    assert data.read_val_dump(str(p))["ch_idx"].shape == (6,)
