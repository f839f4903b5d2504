"""Precompute '.spec.npy' / '.mel.npy' next to every WAV under a directory (reference
prepare_spectrogram.py:13-55), with the HIP featurizer of ``features.py``.

    python prepare_spectrogram.py <path> -c config.json
"""
import argparse
import os
import sys
from glob import glob

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from data_loader import wav_io  # noqa: E402
from features import LogSpectrogram  # noqa: E402
from parse_config import ConfigParser  # noqa: E402


def main(path, config):
    sp = config["spectrogram"]
    window_length = sp.get("window_length", 1024)
    hop_samples = sp["hop_samples"]
    n_mels = config["mel_spectrogram"]["n_mels"] if "mel_spectrogram" in config.config else 128
    sample_rate = config["sample_rate"]
    spec_fn = LogSpectrogram(window_length, hop_samples, mel=False)
    mel_fn = LogSpectrogram(window_length, hop_samples, mel=True, n_mels=n_mels, sample_rate=sample_rate)
    for filename in sorted(glob(f"{path}/**/*.wav", recursive=True)):
        audio, sr = wav_io.load(filename)
        assert sr == sample_rate
        a = audio.cuda()
        np.save(f"{filename}.mel.npy", torch.squeeze(mel_fn(a)).cpu().numpy())
        np.save(f"{filename}.spec.npy", torch.squeeze(spec_fn(a)).cpu().numpy())


if __name__ == "__main__":
    args = argparse.ArgumentParser(description="Speech denoising diffusion model")
    args.add_argument("path", type=str, help="data path")
    args.add_argument("-c", "--config", default=None, type=str, help="config file path")
    args = args.parse_args()
    args.resume = None
    args.device = None
    main(args.path, ConfigParser.from_args(args))
