"""Synthetic VoiceBank-DEMAND-shaped inputs (SURVEY.md §8d "Synthetic inputs").

There is no network and no dataset on the build or GPU boxes, so every bench and
test input is generated here: 16 kHz mono chunks made of a harmonic source
(f0 ~ U[90, 250] Hz, 10 harmonics with 1/k amplitudes, 4 Hz syllabic AM,
RMS 0.05) plus Gaussian noise at an SNR drawn from {2.5, 7.5, 12.5, 17.5} dB,
clipped to [-1, 1] — the noisy ``condition`` the reference's ``infer.py``
feeds to ``model.infer`` (infer.py:72-77).
"""
import numpy as np

SNRS_DB = (2.5, 7.5, 12.5, 17.5)


def noisy_speech(batch, n_samples, seed=1234, sample_rate=16000, return_clean=False):
    rng = np.random.default_rng(seed)
    t = np.arange(n_samples, dtype=np.float64) / sample_rate
    clean = np.empty((batch, n_samples), dtype=np.float64)
    noisy = np.empty((batch, n_samples), dtype=np.float64)
    for b in range(batch):
        f0 = rng.uniform(90.0, 250.0)
        phase = rng.uniform(0, 2 * np.pi, size=10)
        s = sum(np.sin(2 * np.pi * f0 * k * t + phase[k - 1]) / k for k in range(1, 11))
        s *= 0.5 * (1.0 + np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 2 * np.pi)))
        s *= 0.05 / max(np.sqrt(np.mean(s * s)), 1e-12)
        snr = SNRS_DB[rng.integers(len(SNRS_DB))]
        n = rng.standard_normal(n_samples)
        n *= np.sqrt(np.mean(s * s) / 10 ** (snr / 10)) / max(np.sqrt(np.mean(n * n)), 1e-12)
        clean[b] = s
        noisy[b] = np.clip(s + n, -1.0, 1.0)
    noisy = noisy.astype(np.float32).reshape(batch, 1, n_samples)
    if return_clean:
        return noisy, clean.astype(np.float32).reshape(batch, 1, n_samples)
    return noisy
