"""ORACLE (test infrastructure only) — log-magnitude (mel) spectrogram in numpy.

Restates prepare_spectrogram.py:20-55 of the reference, i.e. torchaudio.transforms.Spectrogram
(Hamming window, prepare_spectrogram.py:22) / MelSpectrogram (no window_fn: torchaudio's default
Hann window, prepare_spectrogram.py:27-35), power=1, normalized=True, center=True, reflect
padding, followed by clamp((log10(S) - 1 + 5) / 5, 0, 1).  torchaudio (unpinned by the reference, absent here) is
restated from its published algorithm; float64 rfft.  Parity: pinned against torch.stft-based
fixtures (tests/golden/gen_golden.py --only stft), not against torchaudio itself.
"""
import numpy as np


def hamming(n):
    k = np.arange(n, dtype=np.float64)
    return (0.54 - 0.46 * np.cos(2 * np.pi * k / n)).astype(np.float32)     # periodic=True


def hann(n):
    k = np.arange(n, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2 * np.pi * k / n)).astype(np.float32)       # periodic=True


def magnitude(audio, n_fft=1024, hop=256, window=None):
    """|STFT| / sqrt(sum w^2): audio [B, N] -> [B, n_fft/2+1, 1 + N // hop] (float64)."""
    w = (hamming(n_fft) if window is None else window).astype(np.float64)
    x = np.pad(audio.astype(np.float64), ((0, 0), (n_fft // 2, n_fft // 2)), mode="reflect")
    F = 1 + audio.shape[1] // hop
    idx = np.arange(F)[:, None] * hop + np.arange(n_fft)[None, :]
    spec = np.fft.rfft(x[:, idx] * w, axis=-1)                               # [B, F, bins]
    return np.abs(spec).transpose(0, 2, 1) / np.sqrt(np.sum(w * w))


def log_features(S):
    with np.errstate(divide="ignore"):
        v = np.log10(S) - 1.0
    return np.clip((v + 5.0) / 5.0, 0.0, 1.0).astype(np.float32)


def log_spectrogram(audio, n_fft=1024, hop=256, window=None, fb=None):
    """fb given (mel): the window defaults to Hann, as MelSpectrogram's; else Hamming."""
    if window is None and fb is not None:
        window = hann(n_fft)
    S = magnitude(audio, n_fft, hop, window)
    if fb is not None:
        S = np.einsum("km,bkf->bmf", fb.astype(np.float64), S)
    return log_features(S)
