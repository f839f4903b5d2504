"""Inference data path (reference data_loader/data_loaders.py:13-164): file inventory, chunking of
each file into T-sample pieces (InferDataset), the chunk-concatenating collate and InferDataLoader.

Deviations: WAV I/O through ``wav_io`` (torchaudio is absent), and the inventory is sorted (the
reference keeps ``Path.glob`` order, which the filesystem decides).
"""
from math import ceil
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset

from . import wav_io


def generate_inventory(path, file_type=".wav"):
    """data_loaders.py:13-20."""
    path = Path(path)
    assert path.is_dir(), "{:s} is not a valid directory".format(str(path))
    file_names = sorted(p.name for p in path.glob("*" + file_type))
    assert file_names, "{:s} has no valid {} file".format(str(path), file_type)
    return file_names


class AudioDataset(Dataset):
    """data_loaders.py:23-90 (constructor, length, getName)."""

    def __init__(self, data_root, datatype, sample_rate=8000, T=-1):
        if datatype not in [".wav", ".logwav.npy", ".spec.npy", ".mel.npy"]:
            raise NotImplementedError
        self.datatype = datatype
        self.sample_rate = sample_rate
        self.T = T
        self.clean_path = Path("{}/clean".format(data_root))
        self.noisy_path = Path("{}/noisy".format(data_root))
        self.inventory = generate_inventory(self.clean_path, datatype)
        self.data_len = len(self.inventory)

    def __len__(self):
        return self.data_len

    def getName(self, idx):
        if self.datatype == ".wav":
            return self.inventory[idx].rsplit(".", 1)[0]
        return self.inventory[idx].rsplit(".", 2)[0]


class InferDataset(AudioDataset):
    """data_loaders.py:101-141: one item = every T-sample chunk of one file, zero-padded at the end,
    as (clean [n,1,T], noisy [n,1,T], file index [n])."""

    def __getitem__(self, index):
        if self.datatype == ".wav":
            clean, sr = wav_io.load(self.clean_path / self.inventory[index])
            assert sr == self.sample_rate
            noisy, sr = wav_io.load(self.noisy_path / self.inventory[index])
            assert sr == self.sample_rate
        elif self.datatype == ".logwav.npy":
            clean = torch.from_numpy(np.load(self.clean_path / self.inventory[index]))
            noisy = torch.from_numpy(np.load(self.noisy_path / self.inventory[index]))
        else:
            raise NotImplementedError
        n_frames = clean.shape[-1]
        assert n_frames == noisy.shape[-1]
        n_chunk = ceil(n_frames / self.T)
        clean = F.pad(clean, (0, n_chunk * self.T - n_frames), "constant", 0)
        noisy = F.pad(noisy, (0, n_chunk * self.T - n_frames), "constant", 0)
        index_tensor = index * torch.ones(n_chunk, dtype=torch.long)
        return clean.reshape(n_chunk, 1, self.T), noisy.reshape(n_chunk, 1, self.T), index_tensor


def infer_data_collate(batch):
    """data_loaders.py:143-155: concatenate the chunks of every file of the batch."""
    clean, noisy, index = zip(*batch)
    return torch.cat(clean, dim=0), torch.cat(noisy, dim=0), torch.cat(index, dim=0)


class InferDataLoader(DataLoader):
    """data_loaders.py:158-164 (BaseDataLoader with shuffle=False, validation_split=0)."""

    def __init__(self, dataset, batch_size, num_workers=1):
        self.dataset_ = dataset
        self.n_samples = len(dataset)
        super().__init__(dataset, batch_size=batch_size, shuffle=False, collate_fn=infer_data_collate,
                         num_workers=num_workers)
