"""ORACLE (test infrastructure only) — UNetModified2 forward in numpy.

Restates model/UNetModified2.py of the reference:
  SignalToFrames.forward / overlapAdd   UNetModified2.py:23-41
  PositionalEncoding                    UNetModified2.py:49-68
  FeatureWiseAffine (use_affine_level=False)  UNetModified2.py:72-89
  Upsample / Downsample                 UNetModified2.py:93-109
  Block (GroupNorm -> Swish -> Conv3x3) UNetModified2.py:113-124
  ResnetBlock                           UNetModified2.py:127-142
  UNetModified2.__init__ / forward      UNetModified2.py:146-269

Weights come as a dict of numpy arrays keyed exactly like the reference
``state_dict`` without the ``noise_estimate_model.`` prefix.  Tensors are NCHW
float32 [B, C, H=frames, W=segment_len].  Convolutions are 9 tap-shifted
float32 GEMMs (BLAS sgemm), GroupNorm statistics in float64.
"""
import numpy as np

f32 = np.float32


def embedding_vector(dim):
    """PositionalEncoding.embedding_vector (UNetModified2.py:53-55): fp32
    1e4 * 10 ** (-k * 4 / half).  Pinned bit-exact against the fixture."""
    half = dim // 2
    step = np.arange(half)
    e = (-(step.astype(np.float32)) * f32(4.0)) / f32(half)
    return (f32(1e4) * np.power(f32(10.0), e).astype(np.float32)).astype(np.float32)


def architecture(num_samples, in_channel=2, out_channel=1, inner_channel=32, norm_groups=32,
                 channel_mults=(1, 2, 3, 4, 5), res_blocks=3, dropout=0, segment_len=128,
                 segment_stride=64):
    """Layer list of UNetModified2.__init__ (UNetModified2.py:147-235).

    Returns dict with 'downs', 'mid', 'ups' lists of (kind, name, c_in, c_out)."""
    assert (num_samples - segment_len) % segment_stride == 0          # UNetModified2.py:13
    downs = [("conv", "downs.0", in_channel, inner_channel)]
    feat = [inner_channel]
    cin = inner_channel
    idx = 1
    for ind, mult in enumerate(channel_mults):
        cout = inner_channel * mult
        for _ in range(res_blocks):
            downs.append(("res", f"downs.{idx}", cin, cout)); idx += 1
            feat.append(cout)
            cin = cout
        downs.append(("down", f"downs.{idx}", cout, cout)); idx += 1
        feat.append(cout)
    mid = [("res", "mid.0", cin, cin)]
    ups = []
    idx = 0
    for ind in reversed(range(len(channel_mults))):
        cin = inner_channel * channel_mults[ind]
        cout = cin
        ups.append(("res", f"ups.{idx}", cin + feat.pop(), cout)); idx += 1
        ups.append(("up", f"ups.{idx}", cout, cout)); idx += 1
        cout = inner_channel if ind == 0 else inner_channel * channel_mults[ind - 1]
        for _ in range(res_blocks):
            ups.append(("res", f"ups.{idx}", cin + feat.pop(), cout)); idx += 1
            cin = cout
    final = ("final", "final_conv", cout, out_channel)
    return dict(downs=downs, mid=mid, ups=ups, final=final, groups=norm_groups,
                seg=segment_len, stride=segment_stride, inner=inner_channel)


def frame_index(n_samples, F, stride):
    """SignalToFrames.idx_mat (UNetModified2.py:13-20)."""
    n_frames = (n_samples - F) // stride + 1
    return np.arange(n_frames)[:, None] * stride + np.arange(F)[None, :]


def overlap_add(frames, n_samples, stride):
    """SignalToFrames.overlapAdd (UNetModified2.py:30-41): un-normalised OLA."""
    B, C, nf, F = frames.shape
    out = np.zeros((B, C, n_samples), dtype=np.float32)
    for i in range(nf):
        out[:, :, i * stride:i * stride + F] += frames[:, :, i, :]
    return out


def swish(x):
    """Swish (UNetModified2.py:44-46): x * sigmoid(x)."""
    with np.errstate(over="ignore"):
        return (x * (f32(1.0) / (f32(1.0) + np.exp(-x)))).astype(np.float32)


def group_norm(x, groups, gamma, beta, eps=1e-5):
    """nn.GroupNorm(groups, C) (UNetModified2.py:117): biased variance, eps 1e-5."""
    B, C, H, W = x.shape
    xg = x.reshape(B, groups, -1).astype(np.float64)
    mean = xg.mean(axis=2, keepdims=True)
    var = ((xg - mean) ** 2).mean(axis=2, keepdims=True)
    y = ((xg - mean) / np.sqrt(var + eps)).reshape(B, C, H, W)
    return (y * gamma[None, :, None, None] + beta[None, :, None, None]).astype(np.float32)


def conv2d(x, w, b, stride=1):
    """nn.Conv2d(k=3, pad=1, stride) or k=1 as tap-shifted GEMMs."""
    B, C, H, W = x.shape
    co, ci, kh, kw = w.shape
    if kh == 1:   # per batch row, so results do not depend on how rows are batched / sharded
        w2 = np.ascontiguousarray(w[:, :, 0, 0])
        out = np.stack([(w2 @ x[i].reshape(C, H * W)).reshape(co, H, W) for i in range(B)])
        return (out + b[None, :, None, None]).astype(np.float32)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    wm = np.ascontiguousarray(w.transpose(0, 2, 3, 1).reshape(co, 9 * C))   # k = (tap, ci)
    out = np.empty((B, co, Ho * Wo), dtype=np.float32)
    cols = np.empty((9, C, Ho, Wo), dtype=np.float32)
    for bi in range(B):                                  # one im2col GEMM per batch row
        xp = np.zeros((C, H + 2, W + 2), dtype=np.float32)
        xp[:, 1:-1, 1:-1] = x[bi]
        for dy in range(3):
            for dx in range(3):
                cols[dy * 3 + dx] = xp[:, dy:dy + stride * (Ho - 1) + 1:stride, dx:dx + stride * (Wo - 1) + 1:stride]
        out[bi] = wm @ cols.reshape(9 * C, Ho * Wo)
    return (out.reshape(B, co, Ho, Wo) + b[None, :, None, None]).astype(np.float32)


def linear(x, w, b):
    """nn.Linear, row by row (batch-invariant rounding)."""
    return np.stack([w @ xi + b for xi in x]).astype(np.float32)


def noise_level_embedding(P, noise_level, inner):
    """noise_level_mlp (UNetModified2.py:168-174, 249): PositionalEncoding in fp32
    (product rounded to fp32, sin/cos accurate), Linear-Swish-Linear-Swish."""
    ev = embedding_vector(inner)
    arg = (np.asarray(noise_level, dtype=np.float32).reshape(-1, 1) * ev[None, :]).astype(np.float32)
    enc = np.concatenate([np.sin(arg.astype(np.float64)), np.cos(arg.astype(np.float64))], -1).astype(np.float32)
    h = swish(linear(enc, P["noise_level_mlp.1.weight"], P["noise_level_mlp.1.bias"]))
    return swish(linear(h, P["noise_level_mlp.3.weight"], P["noise_level_mlp.3.bias"]))


def block(P, name, x, groups):
    """Block (UNetModified2.py:113-124): GN -> Swish -> Conv3x3."""
    h = swish(group_norm(x, groups, P[f"{name}.block.0.weight"], P[f"{name}.block.0.bias"]))
    return conv2d(h, P[f"{name}.block.3.weight"], P[f"{name}.block.3.bias"])


def resnet_block(P, name, x, temb, groups, cin, cout):
    """ResnetBlock (UNetModified2.py:127-142)."""
    h = block(P, f"{name}.block1", x, groups)
    lin = linear(temb, P[f"{name}.noise_func.noise_func.0.weight"], P[f"{name}.noise_func.noise_func.0.bias"])
    h = (h + lin[:, :, None, None]).astype(np.float32)
    h = block(P, f"{name}.block2", h, groups)
    if cin != cout:
        r = conv2d(x, P[f"{name}.res_conv.weight"], P[f"{name}.res_conv.bias"])
    else:
        r = x
    return (h + r).astype(np.float32)


def forward(P, arch, cond, x_t, noise_level):
    """UNetModified2.forward (UNetModified2.py:237-269).

    cond, x_t: [B, 1, N] float32; noise_level: [B] float32.  Returns [B, 1, N]."""
    N = cond.shape[-1]
    idx = frame_index(N, arch["seg"], arch["stride"])
    x = np.concatenate([cond[:, :, idx], x_t[:, :, idx]], axis=1).astype(np.float32)   # :244-247
    t = noise_level_embedding(P, noise_level, arch["inner"])                             # :249
    G = arch["groups"]
    feats = []
    for kind, name, ci, co in arch["downs"]:                                             # :252-257
        if kind == "res":
            x = resnet_block(P, name, x, t, G, ci, co)
        elif kind == "down":
            x = conv2d(x, P[f"{name}.conv.weight"], P[f"{name}.conv.bias"], stride=2)
        else:
            x = conv2d(x, P[f"{name}.weight"], P[f"{name}.bias"])
        feats.append(x)
    for kind, name, ci, co in arch["mid"]:                                               # :258-259
        x = resnet_block(P, name, x, t, G, ci, co)
    for kind, name, ci, co in arch["ups"]:                                               # :261-265
        if kind == "res":
            x = resnet_block(P, name, np.concatenate([x, feats.pop()], axis=1), t, G, ci, co)
        else:
            x = np.repeat(np.repeat(x, 2, axis=2), 2, axis=3)
            x = conv2d(x, P[f"{name}.conv.weight"], P[f"{name}.conv.bias"])
    y = block(P, "final_conv", x, G)                                                     # :267
    return overlap_add(y, N, arch["stride"])                                             # :268
