"""GPU: the spectrogram featurizer (reference prepare_spectrogram.py:20-55) through
features.LogSpectrogram and sddm_log_spectrogram, against the torch.stft-based fixture and the
numpy oracle at the DiffWave clip length."""
import numpy as np
import pytest
import torch

from _helpers import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mel", [False, True])
def test_log_spectrogram_matches_fixture(torch_cuda, mel):
    from features import LogSpectrogram
    z = golden("stft.npz")
    f = LogSpectrogram(1024, 256, mel=mel, n_mels=128, sample_rate=16000)
    # prepare_spectrogram.py: Hamming for the linear spectrogram, MelSpectrogram's default Hann for mel
    assert np.abs(f.window.numpy() - z["stft/window_mel" if mel else "stft/window"]).max() == 0
    assert np.abs(f.window.numpy() - (np.hanning(1025)[:-1] if mel else np.hamming(1025)[:-1])).max() < 1e-6
    if mel:
        assert np.abs(f.fb.numpy() - z["stft/fb"]).max() == 0
    out = f(torch.from_numpy(z["stft/audio"]).cuda()).cpu().numpy()
    ref = z["stft/mel" if mel else "stft/spec"]
    assert out.shape == ref.shape
    assert np.abs(out - ref).max() <= 1e-4


def test_log_spectrogram_full_clip_matches_oracle(torch_cuda):
    from features import LogSpectrogram
    from oracle import features as fe
    from sddm_hip.synth import noisy_speech
    audio = noisy_speech(3, 16128, seed=8).reshape(3, -1).astype(np.float32)
    f = LogSpectrogram(1024, 256)
    out = f(torch.from_numpy(audio).cuda()).cpu().numpy()
    ref = fe.log_spectrogram(audio, window=f.window.numpy())
    assert out.shape == (3, 513, 64)
    assert np.abs(out - ref).max() <= 1e-4


def test_prepare_spectrogram_cli_writes_features(torch_cuda, tmp_path):
    import prepare_spectrogram
    from data_loader import wav_io
    from parse_config import ConfigParser
    wav_io.save(tmp_path / "a.wav", torch.sin(torch.arange(5000) * 0.03)[None] * 0.3, 16000)
    cfg = {"name": "p", "sample_rate": 16000, "spectrogram": {"window_length": 1024, "hop_samples": 256},
           "mel_spectrogram": {"n_mels": 128}, "trainer": {"save_dir": None}}
    prepare_spectrogram.main(str(tmp_path), ConfigParser(cfg))
    assert np.load(tmp_path / "a.wav.spec.npy").shape == (513, 1 + 5000 // 256)
    assert np.load(tmp_path / "a.wav.mel.npy").shape == (128, 1 + 5000 // 256)
