"""Minimal WAV reader/writer (torchaudio is not available in this image).

``load`` mirrors ``torchaudio.load``'s default: a float32 tensor [channels, frames] normalised to
[-1, 1) for integer PCM (divide by 2^(bits-1)), IEEE-float data unchanged, and the sample rate.
``save`` mirrors ``torchaudio.save`` of a float32 tensor: a 32-bit IEEE-float WAV (format tag 3).
"""
import struct

import numpy as np
import torch


def load(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:                  # WAVE_FORMAT_EXTENSIBLE
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, sr, bits = fmt
    if tag == 3 and bits == 32:
        x = np.frombuffer(pcm, "<f4").astype(np.float32)
    elif tag == 3 and bits == 64:
        x = np.frombuffer(pcm, "<f8").astype(np.float32)
    elif tag == 1 and bits == 16:
        x = np.frombuffer(pcm, "<i2").astype(np.float32) / 32768.0
    elif tag == 1 and bits == 32:
        x = (np.frombuffer(pcm, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    elif tag == 1 and bits == 8:
        x = (np.frombuffer(pcm, "u1").astype(np.float32) - 128.0) / 128.0
    else:
        raise NotImplementedError(f"{path}: WAV format tag {tag} with {bits} bits")
    x = x[: len(x) // ch * ch].reshape(-1, ch).T.copy()
    return torch.from_numpy(x), sr


def save(path, tensor, sample_rate):
    x = tensor.detach().cpu().float().numpy()
    if x.ndim == 1:
        x = x[None]
    ch = x.shape[0]
    pcm = np.ascontiguousarray(x.T).astype("<f4").tobytes()
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + len(pcm), b"WAVE", b"fmt ", 16, 3, ch, int(sample_rate),
                      int(sample_rate) * 4 * ch, 4 * ch, 32, b"data", len(pcm))
    with open(path, "wb") as f:
        f.write(hdr + pcm)
