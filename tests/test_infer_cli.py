"""CPU: the inference data path around the hot path -- WAV I/O,
InferDataset chunking / collate / regrouping (data_loaders.py:101-164, infer.py:70-126), the
checkpoint reader (base_trainer.py:108-128) and SI-SNR (model/metric.py:5-34)."""
import os
import pathlib
import struct

import numpy as np
import pytest
import torch


def _write_pcm16(path, x, sr=16000):
    pcm = np.clip(np.round(x * 32768), -32768, 32767).astype("<i2").tobytes()
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(pcm), b"WAVE", b"fmt ", 16, 1, 1, sr, 2 * sr, 2, 16,
                      b"data", len(pcm))
    with open(path, "wb") as f:
        f.write(hdr + pcm)


def test_wav_float_roundtrip_and_pcm16_scaling(tmp_path):
    from data_loader import wav_io
    x = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, (1, 1000)).astype(np.float32))
    wav_io.save(tmp_path / "a.wav", x, 16000)
    y, sr = wav_io.load(tmp_path / "a.wav")
    assert sr == 16000 and torch.equal(x, y)
    _write_pcm16(tmp_path / "b.wav", np.array([0.5, -1.0, 0.25]))
    y, _ = wav_io.load(tmp_path / "b.wav")
    assert y.tolist() == [[0.5, -1.0, 0.25]]


def _dataset(tmp_path, lengths, T):
    from data_loader import data_loaders as D
    rng = np.random.default_rng(1)
    for d in ("clean", "noisy"):
        os.makedirs(tmp_path / d, exist_ok=True)
    for i, n in enumerate(lengths):
        c = rng.uniform(-0.5, 0.5, n)
        _write_pcm16(tmp_path / "clean" / f"f{i}.wav", c)
        _write_pcm16(tmp_path / "noisy" / f"f{i}.wav", c + rng.uniform(-0.1, 0.1, n))
    return D.InferDataset(str(tmp_path), ".wav", sample_rate=16000, T=T)


def test_infer_dataset_chunks_pad_and_index(tmp_path):
    T = 2112
    ds = _dataset(tmp_path, [5000, 2112, 100], T)
    assert len(ds) == 3 and ds.getName(0) == "f0"
    clean, noisy, idx = ds[0]
    assert clean.shape == (3, 1, T) and noisy.shape == (3, 1, T)      # ceil(5000 / 2112) = 3
    assert idx.tolist() == [0, 0, 0]
    flat = noisy.reshape(-1)
    assert torch.all(flat[5000:] == 0) and torch.any(flat[:5000] != 0)
    assert ds[1][0].shape == (1, 1, T) and ds[2][0].shape == (1, 1, T)


def test_collate_and_regroup_flush_every_file(tmp_path):
    from data_loader import data_loaders as D
    import infer
    ds = _dataset(tmp_path, [5000, 2112, 100], 2112)
    clean, noisy, idx = D.infer_data_collate([ds[0], ds[1], ds[2]])
    assert clean.shape == (5, 1, 2112) and idx.tolist() == [0, 0, 0, 1, 2]
    assert infer.regroup(idx) == [(0, [0, 1, 2]), (1, [3]), (2, [4])]   # last file kept


class _Identity:
    def infer(self, condition, **kw):
        return condition.clone()


def test_run_writes_every_file_stitched(tmp_path):
    from data_loader import data_loaders as D, wav_io
    from parse_config import ConfigParser
    import infer
    ds = _dataset(tmp_path / "data", [5000, 2112, 100], 2112)
    loader = D.InferDataLoader(ds, batch_size=2, num_workers=0)
    cfg = {"name": "t", "sample_rate": 16000, "num_samples": 2112, "loss": "l1_loss",
           "trainer": {"save_dir": str(tmp_path / "out")}}
    config = ConfigParser(cfg, run_id="r")
    log = infer.run(config, _Identity(), loader, ds, torch.device("cpu"))
    for i in range(3):
        out, sr = wav_io.load(pathlib.Path(config.save_dir) / "samples" / "output" / f"f{i}.wav")
        noisy = ds[i][1].reshape(1, -1)
        assert sr == 16000 and torch.equal(out, noisy)
    assert np.isfinite(log["loss"]) and np.isfinite(log["sisnr"])


class _FakeConfig:          # stands in for the reference ConfigParser pickled into checkpoints
    def __init__(self):
        self._config = {"name": "x"}
        self.resume = pathlib.Path("/tmp/somewhere")

    def __setstate__(self, state):     # never called by the reader
        raise AssertionError("checkpoint object was executed")


def test_checkpoint_reader_loads_weights_without_executing_objects(tmp_path):
    from checkpoint import load_checkpoint, state_dict_from_checkpoint
    sd = {"module.noise_estimate_model.w": torch.arange(6.0).reshape(2, 3), "module.diffusion.betas": torch.ones(4)}
    path = tmp_path / "ck.pth"
    torch.save({"arch": "SDDM", "epoch": 3, "state_dict": sd, "optimizer": {"state": {}, "param_groups": []},
                "monitor_best": 0.5, "config": _FakeConfig()}, path)
    ck = load_checkpoint(str(path))
    assert ck["epoch"] == 3 and type(ck["config"]).__name__ == "_FakeConfig"
    got = state_dict_from_checkpoint(str(path))
    assert set(got) == {"noise_estimate_model.w", "diffusion.betas"}
    assert torch.equal(got["noise_estimate_model.w"], sd["module.noise_estimate_model.w"])


def test_sisnr_matches_definition():
    from model.metric import sisnr
    rng = np.random.default_rng(2)
    s = rng.standard_normal((3, 1, 400))
    s_hat = s + 0.1 * rng.standard_normal((3, 1, 400))
    v = float(sisnr(torch.from_numpy(s_hat), torch.from_numpy(s)))
    ref = []
    for a, b in zip(s_hat[:, 0], s[:, 0]):
        a, b = a - a.mean(), b - b.mean()
        st = (a @ b) * b / (b @ b)
        ref.append(10 * np.log10((st @ st) / ((a - st) @ (a - st))))
    assert v == pytest.approx(np.mean(ref), rel=1e-9)


def test_run_logwav_npy_reverses_log_modulus(tmp_path):
    """'.logwav.npy' data (data_loaders.py:125-139) are stitched and mapped back through
    log_modulus_normalize_reverse (infer.py:104-116, prepare_logaudio.py:22-26)."""
    from data_loader import data_loaders as D, wav_io
    from parse_config import ConfigParser
    import infer
    rng = np.random.default_rng(5)
    for d in ("clean", "noisy"):
        os.makedirs(tmp_path / "data" / d)
    x = rng.uniform(-0.5, 0.5, (1, 3000)).astype(np.float32)
    np.save(tmp_path / "data" / "clean" / "g.logwav.npy", x)
    np.save(tmp_path / "data" / "noisy" / "g.logwav.npy", x)
    ds = D.InferDataset(str(tmp_path / "data"), ".logwav.npy", sample_rate=16000, T=2112)
    assert ds.getName(0) == "g"
    loader = D.InferDataLoader(ds, batch_size=1, num_workers=0)
    config = ConfigParser({"name": "l", "sample_rate": 16000, "num_samples": 2112, "loss": "l1_loss",
                           "trainer": {"save_dir": str(tmp_path / "out")}}, run_id="r")
    infer.run(config, _Identity(), loader, ds, torch.device("cpu"))
    out, _ = wav_io.load(pathlib.Path(config.save_dir) / "samples" / "output" / "g.wav")
    padded = torch.from_numpy(np.pad(x, ((0, 0), (0, 2 * 2112 - 3000))))
    assert torch.allclose(out, infer.log_modulus_normalize_reverse(padded, 3), rtol=0, atol=0)
