"""ORACLE (test infrastructure only) — DiffWave forward in numpy (float32).

Restates model/diffwave.py of the reference:
  DiffusionEmbedding (embedding_vector 10 ** ((k/64) * 4/63))  diffwave.py:22-45
  SpectrogramUpsampler (2 x ConvTranspose2d [3,32] stride [1,16] pad [1,8] + leaky_relu 0.4)
                                                                         diffwave.py:48-61
  ResidualBlock (split=True: output_residual + output_projection)         diffwave.py:64-108
  DiffWave.forward                                                        diffwave.py:133-155

Weights: dict of numpy arrays keyed like the reference state_dict without the
``noise_estimate_model.`` prefix.  Activations are [B, C, N] float32; every 1x1 / dilated
Conv1d is a float32 GEMM over the channel axis.
"""
import numpy as np

f32 = np.float32


def embedding_vector(dim=128):
    """DiffusionEmbedding.embedding_vector (diffwave.py:25-28) with torch's fp32 op order."""
    half = dim // 2
    step = (np.arange(half, dtype=np.float32) / f32(half)).astype(np.float32)
    e = ((step * f32(4.0)).astype(np.float32) / f32(63)).astype(np.float32)
    return np.power(f32(10.0), e).astype(np.float32)


def _silu(x):
    return (x * (f32(1.0) / (f32(1.0) + np.exp(-x)))).astype(np.float32)


def embedding(P, steps):
    """DiffusionEmbedding.forward (diffwave.py:32-45): steps [B] -> [B, 512]."""
    enc = (steps.astype(np.float32)[:, None] * embedding_vector()[None, :]).astype(np.float32)
    x = np.concatenate([np.sin(enc), np.cos(enc)], axis=-1).astype(np.float32)
    x = _silu(x @ P["diffusion_embedding.projection1.weight"].T + P["diffusion_embedding.projection1.bias"])
    x = _silu(x @ P["diffusion_embedding.projection2.weight"].T + P["diffusion_embedding.projection2.bias"])
    return x


def conv_transpose_time(x, k, bias):
    """ConvTranspose2d(1, 1, [3, 32], stride=[1, 16], padding=[1, 8]) on [B, H, W]
    (diffwave.py:51-52): out[h, w] = bias + sum in[hi, wi] * k[kh, kw], h = hi - 1 + kh,
    w = 16 wi - 8 + kw."""
    B, H, W = x.shape
    Wo = 16 * W
    out = np.zeros((B, H + 2, 16 * W + 32), dtype=np.float32)   # padded canvas
    for kh in range(3):
        for kw in range(32):
            # h index in canvas = hi + kh (offset 1), w index = 16 wi + kw (offset 8)
            out[:, kh:kh + H, kw:kw + 16 * W:16] += x * k[kh, kw]
    return (out[:, 1:1 + H, 8:8 + Wo] + bias).astype(np.float32)


def _leaky(x, s=0.4):
    return np.where(x > 0, x, (x * f32(s)).astype(np.float32)).astype(np.float32)


def upsample(P, spec):
    """SpectrogramUpsampler.forward (diffwave.py:54-61): [B, bins, F] -> [B, bins, 256 F]."""
    x = _leaky(conv_transpose_time(spec, P["spectrogram_upsampler.conv1.weight"][0, 0],
                                   P["spectrogram_upsampler.conv1.bias"][0]))
    return _leaky(conv_transpose_time(x, P["spectrogram_upsampler.conv2.weight"][0, 0],
                                      P["spectrogram_upsampler.conv2.bias"][0]))


def conv1x1(x, w, b):
    """Conv1d(k=1) on [B, Cin, N] with weight [Cout, Cin, 1]."""
    return (np.einsum("oc,bcn->bon", w[:, :, 0], x, optimize=True) + b[None, :, None]).astype(np.float32)


def dilated_conv(x, w, b, d):
    """Conv1d(C, 2C, 3, padding=d, dilation=d) on [B, C, N] (zero padding of its input)."""
    B, C, N = x.shape
    xp = np.zeros((B, C, N + 2 * d), dtype=np.float32)
    xp[:, :, d:d + N] = x
    y = np.zeros((B, w.shape[0], N), dtype=np.float32)
    for k in range(3):
        y += np.einsum("oc,bcn->bon", w[:, :, k], xp[:, :, k * d:k * d + N], optimize=True)
    return (y + b[None, :, None]).astype(np.float32)


def forward(P, spec, audio, steps, residual_layers=30, cycle=10):
    """DiffWave.forward (diffwave.py:133-155): spec [B, bins, F], audio [B, 1, N], steps [B]."""
    x = np.maximum(conv1x1(audio.astype(np.float32), P["input_projection.weight"], P["input_projection.bias"]), 0)
    emb = embedding(P, steps)
    up = upsample(P, spec.astype(np.float32))
    skip = None
    for i in range(residual_layers):
        p = f"residual_layers.{i}."
        ds = (emb @ P[p + "diffusion_projection.weight"].T + P[p + "diffusion_projection.bias"]).astype(np.float32)
        cond = conv1x1(up, P[p + "conditioner_projection.weight"], P[p + "conditioner_projection.bias"])
        y = (x + ds[:, :, None]).astype(np.float32)
        y = dilated_conv(y, P[p + "dilated_conv.weight"], P[p + "dilated_conv.bias"], 2 ** (i % cycle)) + cond
        C = y.shape[1] // 2
        gate, filt = y[:, :C], y[:, C:]
        y = ((f32(1.0) / (f32(1.0) + np.exp(-gate))) * np.tanh(filt)).astype(np.float32)
        res = conv1x1(y, P[p + "output_residual.weight"], P[p + "output_residual.bias"])
        sk = conv1x1(y, P[p + "output_projection.weight"], P[p + "output_projection.bias"])
        x = ((x + res) / f32(np.sqrt(2.0))).astype(np.float32)
        skip = sk if skip is None else (skip + sk).astype(np.float32)
    x = (skip / f32(np.sqrt(residual_layers))).astype(np.float32)
    x = np.maximum(conv1x1(x, P["skip_projection.weight"], P["skip_projection.bias"]), 0)
    return conv1x1(x, P["output_projection.weight"], P["output_projection.bias"])


def param_shapes(bins=513, C=64, layers=30):
    """State-dict shapes of DiffWave (diffwave.py:113-131) without the module prefix."""
    s = {"input_projection.weight": (C, 1, 1), "input_projection.bias": (C,),
         "diffusion_embedding.projection1.weight": (512, 128), "diffusion_embedding.projection1.bias": (512,),
         "diffusion_embedding.projection2.weight": (512, 512), "diffusion_embedding.projection2.bias": (512,),
         "spectrogram_upsampler.conv1.weight": (1, 1, 3, 32), "spectrogram_upsampler.conv1.bias": (1,),
         "spectrogram_upsampler.conv2.weight": (1, 1, 3, 32), "spectrogram_upsampler.conv2.bias": (1,)}
    for i in range(layers):
        p = f"residual_layers.{i}."
        s[p + "dilated_conv.weight"] = (2 * C, C, 3)
        s[p + "dilated_conv.bias"] = (2 * C,)
        s[p + "diffusion_projection.weight"] = (C, 512)
        s[p + "diffusion_projection.bias"] = (C,)
        s[p + "conditioner_projection.weight"] = (2 * C, bins, 1)
        s[p + "conditioner_projection.bias"] = (2 * C,)
        s[p + "output_projection.weight"] = (C, C, 1)
        s[p + "output_projection.bias"] = (C,)
        s[p + "output_residual.weight"] = (C, C, 1)
        s[p + "output_residual.bias"] = (C,)
    s["skip_projection.weight"] = (C, C, 1)
    s["skip_projection.bias"] = (C,)
    s["output_projection.weight"] = (1, C, 1)
    s["output_projection.bias"] = (1,)
    return s
