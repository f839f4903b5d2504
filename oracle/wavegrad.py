"""ORACLE (test infrastructure only) — WaveGrad forward in numpy.

Restates model/wavegrad.py of the reference:
  PositionalEncoding (exp(-ln(1e4) k / count), sin | cos, added per channel)  wavegrad.py:20-49
  FiLM (input_conv -> leaky 0.2 -> + encoding -> output_conv -> shift | scale) wavegrad.py:52-71
  UBlock (nearest x factor, block1 1x1, block2 / block3 dilated convs + FiLM) wavegrad.py:74-112
  DBlock (residual_dense 1x1 then nearest / factor; 3 leaky + dilated convs)  wavegrad.py:115-137
  WaveGrad.forward                                                           wavegrad.py:167-179

Weights: dict of numpy arrays keyed like the reference state_dict without the
``noise_estimate_model.`` prefix.  Activations are [B, C, N]; every conv accumulates in float64
and rounds to float32 per layer (the reference runs fp32 oneDNN convolutions).
F.interpolate(mode='nearest') with exact integer factors is np.repeat (up) / a stride (down).
"""
import math

import numpy as np

f32 = np.float32

DOWN = [(1, 32, None), (32, 128, 2), (128, 128, 2), (128, 256, 3), (256, 512, 5)]   # wavegrad.py:143-149
FILM = [(32, 128), (128, 128), (128, 256), (256, 512), (512, 512)]                  # wavegrad.py:150-156
UP = [(768, 512, 5, (1, 2, 1, 2)), (512, 512, 5, (1, 2, 1, 2)), (512, 256, 3, (1, 2, 4, 8)),
      (256, 128, 2, (1, 2, 4, 8)), (128, 128, 2, (1, 2, 4, 8))]                     # wavegrad.py:157-163
HOP = 300   # 5 * 5 * 3 * 2 * 2 (config_wavegrad.json hop_samples)


def conv1d(x, w, b, dil=1):
    """Conv1d(Cin, Cout, K, padding=dil*(K-1)/2, dilation=dil) on [B, Cin, N] (same length)."""
    B, C, N = x.shape
    K = w.shape[2]
    pad = dil * (K - 1) // 2
    xp = np.zeros((B, C, N + 2 * pad), dtype=np.float64)
    xp[:, :, pad:pad + N] = x
    y = np.zeros((B, w.shape[0], N), dtype=np.float64)
    for k in range(K):
        y += np.matmul(w[:, :, k].astype(np.float64), xp[:, :, k * dil:k * dil + N])
    return (y + b[None, :, None]).astype(np.float32)


def leaky(x, s=0.2):
    return np.where(x > 0, x, (x * f32(s)).astype(np.float32)).astype(np.float32)


def up(x, f):
    return np.repeat(x, f, axis=2)


def down(x, f):
    return np.ascontiguousarray(x[:, :, ::f][:, :, :x.shape[2] // f])


def encoding_vector(dim):
    """exp(-ln(1e4) * arange(count)/count) in float32 (wavegrad.py:44-47)."""
    count = dim // 2
    step = (np.arange(count, dtype=np.float32) / f32(count)).astype(np.float32)
    return np.exp((f32(-math.log(1e4)) * step).astype(np.float32)).astype(np.float32)


def encoding(noise_level, dim):
    """PositionalEncoding._build_encoding (wavegrad.py:44-49): [B] -> [B, dim]."""
    e = (noise_level.astype(np.float32)[:, None] * encoding_vector(dim)[None, :]).astype(np.float32)
    return np.concatenate([np.sin(e), np.cos(e)], axis=-1).astype(np.float32)


def film(P, i, x, noise_level):
    p = f"film.{i}."
    h = leaky(conv1d(x, P[p + "input_conv.weight"], P[p + "input_conv.bias"]))
    h = (h + encoding(noise_level, x.shape[1])[:, :, None]).astype(np.float32)
    y = conv1d(h, P[p + "output_conv.weight"], P[p + "output_conv.bias"])
    c = y.shape[1] // 2
    return y[:, :c], y[:, c:]


def dblock(P, i, x, f):
    p = f"downsample.{i}."
    res = down(conv1d(x, P[p + "residual_dense.weight"], P[p + "residual_dense.bias"]), f)
    x = down(x, f)
    for j, d in enumerate((1, 2, 4)):
        x = conv1d(leaky(x), P[p + f"conv.{j}.weight"], P[p + f"conv.{j}.bias"], d)
    return (x + res).astype(np.float32)


def ublock(P, i, x, shift, scale, f, dil):
    p = f"upsample.{i}."
    b1 = conv1d(up(x, f), P[p + "block1.weight"], P[p + "block1.bias"])
    b2 = conv1d(up(leaky(x), f), P[p + "block2.0.weight"], P[p + "block2.0.bias"], dil[0])
    b2 = leaky((shift + (scale * b2).astype(np.float32)).astype(np.float32))
    b2 = conv1d(b2, P[p + "block2.1.weight"], P[p + "block2.1.bias"], dil[1])
    x = (b1 + b2).astype(np.float32)
    b3 = leaky((shift + (scale * x).astype(np.float32)).astype(np.float32))
    b3 = conv1d(b3, P[p + "block3.0.weight"], P[p + "block3.0.bias"], dil[2])
    b3 = leaky((shift + (scale * b3).astype(np.float32)).astype(np.float32))
    b3 = conv1d(b3, P[p + "block3.1.weight"], P[p + "block3.1.bias"], dil[3])
    return (x + b3).astype(np.float32)


def forward(P, spec, audio, noise_level):
    """WaveGrad.forward (wavegrad.py:167-179): spec [B, 128, F], audio [B, N=300F], noise [B] ->
    [B, N] (the reference then squeezes; the SDDM_spectrogram adapter of SURVEY Q4 keeps [B, 1, N])."""
    x = audio.astype(np.float32)[:, None, :]
    films = []
    for i, (_, _, f) in enumerate(DOWN):
        if f is None:
            x = conv1d(x, P["downsample.0.weight"], P["downsample.0.bias"])
        else:
            x = dblock(P, i, x, f)
        films.append(film(P, i, x, noise_level))
    x = conv1d(spec.astype(np.float32), P["first_conv.weight"], P["first_conv.bias"])
    for i, (_, _, f, dil) in enumerate(UP):
        shift, scale = films[len(films) - 1 - i]
        x = ublock(P, i, x, shift, scale, f, dil)
    return conv1d(x, P["last_conv.weight"], P["last_conv.bias"])[:, 0]


def param_shapes():
    """State-dict shapes of WaveGrad (wavegrad.py:140-165) without the module prefix."""
    s = {"downsample.0.weight": (32, 1, 5), "downsample.0.bias": (32,)}
    for i, (ci, co, f) in enumerate(DOWN[1:], 1):
        p = f"downsample.{i}."
        s[p + "residual_dense.weight"], s[p + "residual_dense.bias"] = (co, ci, 1), (co,)
        for j, c in enumerate((ci, co, co)):
            s[p + f"conv.{j}.weight"], s[p + f"conv.{j}.bias"] = (co, c, 3), (co,)
    for i, (ci, co) in enumerate(FILM):
        p = f"film.{i}."
        s[p + "input_conv.weight"], s[p + "input_conv.bias"] = (ci, ci, 3), (ci,)
        s[p + "output_conv.weight"], s[p + "output_conv.bias"] = (2 * co, ci, 3), (2 * co,)
    for i, (ci, h, f, _) in enumerate(UP):
        p = f"upsample.{i}."
        s[p + "block1.weight"], s[p + "block1.bias"] = (h, ci, 1), (h,)
        s[p + "block2.0.weight"], s[p + "block2.0.bias"] = (h, ci, 3), (h,)
        for k in ("block2.1", "block3.0", "block3.1"):
            s[p + k + ".weight"], s[p + k + ".bias"] = (h, h, 3), (h,)
    s["first_conv.weight"], s["first_conv.bias"] = (768, 128, 3), (768,)
    s["last_conv.weight"], s["last_conv.bias"] = (1, 128, 3), (1,)
    return s
