"""Spectrogram featurizer on the HIP device (reference prepare_spectrogram.py:13-55).

The reference computes ``torchaudio.transforms.Spectrogram(n_fft=window_length, hop_length=
hop_samples, window_fn=torch.hamming_window, power=1, normalized=True)`` and the matching
``MelSpectrogram(f_min=20, f_max=sr/2, n_mels, power=1, normalized=True)`` -- which passes no
window_fn, so its STFT uses torchaudio's default Hann window (prepare_spectrogram.py:27-35) --
and stores
``clamp((log10(S) - 1 + 5) / 5, 0, 1)``.  torchaudio is not installed here (and its version is
not pinned by the reference); its published algorithm is restated: torch.stft with
``center=True, pad_mode='reflect', onesided=True``, division by ``sqrt(sum(window**2))``
("window" normalisation), magnitude; the mel filterbank is ``melscale_fbanks`` with the HTK mel
scale and no normalisation.  The window and filterbank are built here with torch's fp32 ops;
the per-frame DFT, magnitude, mel projection and log / clamp run in one HIP kernel
(csrc/stft.hip, ``sddm_log_spectrogram``).
"""
import math

import torch

import sddm_hip


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """torchaudio.functional.melscale_fbanks(mel_scale='htk', norm=None): [n_freqs, n_mels]."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + (f_min / 700.0))
    m_max = 2595.0 * math.log10(1.0 + (f_max / 700.0))
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down_slopes = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up_slopes = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down_slopes, up_slopes))


class LogSpectrogram:
    """Callable featurizer: audio [B, N] (or [N]) fp32 on the HIP device -> [B, bins, 1 + N // hop]
    (``mel=False``: bins = n_fft/2 + 1 as in '.spec.npy'; ``mel=True``: n_mels as in '.mel.npy')."""

    def __init__(self, window_length=1024, hop_samples=256, mel=False, n_mels=128, sample_rate=16000, f_min=20.0):
        self.n_fft, self.hop, self.mel = int(window_length), int(hop_samples), bool(mel)
        # '.spec.npy': Hamming (prepare_spectrogram.py:22); '.mel.npy': MelSpectrogram's default Hann
        self.window = torch.hann_window(self.n_fft) if self.mel else torch.hamming_window(self.n_fft)
        self.fb = melscale_fbanks(self.n_fft // 2 + 1, f_min, sample_rate / 2.0, n_mels, sample_rate) if mel else None
        self.n_out = n_mels if mel else self.n_fft // 2 + 1
        self._dev = {}

    def _on(self, device):
        if device not in self._dev:
            self._dev[device] = (self.window.to(device), None if self.fb is None else self.fb.contiguous().to(device))
        return self._dev[device]

    @torch.no_grad()
    def __call__(self, audio):
        if not audio.is_cuda:
            raise RuntimeError("LogSpectrogram runs on the HIP device; move the audio to cuda")
        x = audio.reshape(-1, audio.shape[-1]).contiguous().float()
        w, fb = self._on(x.device)
        out = torch.empty((x.shape[0], self.n_out, 1 + x.shape[1] // self.hop), dtype=torch.float32, device=x.device)
        sddm_hip.log_spectrogram(x, self.n_fft, self.hop, w, fb, self.n_out, out)
        return out
