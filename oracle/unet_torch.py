"""ORACLE (test infrastructure only) — UNetModified2 forward in PyTorch CPU ops.

The same restatement of the reference as oracle/unet.py (UNetModified2.py:23-269, see there for
the line map), expressed with torch's CPU kernels (oneDNN convolutions, native GroupNorm) the way
the reference itself runs on a CPU, so that bench.py's ``cpu_baseline`` times a CPU path of the
reference's speed class rather than the numpy GEMM restatement.  Parity: pinned against the
reference-generated goldens and the numpy oracle by tests/test_oracle.py.  Only tests/ and
bench.py's cpu_baseline leg use it; the product path never imports oracle/.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .unet import embedding_vector, frame_index


def _t(P):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in P.items()}


def _swish(x):
    return x * torch.sigmoid(x)                              # Swish, UNetModified2.py:44-46


def _block(T, name, x, groups):
    """Block (UNetModified2.py:113-124): GroupNorm -> Swish -> Conv3x3 (Dropout p=0)."""
    h = _swish(F.group_norm(x, groups, T[f"{name}.block.0.weight"], T[f"{name}.block.0.bias"], 1e-5))
    return F.conv2d(h, T[f"{name}.block.3.weight"], T[f"{name}.block.3.bias"], padding=1)


def _resnet(T, name, x, temb, groups, cin, cout):
    """ResnetBlock (UNetModified2.py:127-142) with FeatureWiseAffine (:72-89)."""
    h = _block(T, f"{name}.block1", x, groups)
    h = h + F.linear(temb, T[f"{name}.noise_func.noise_func.0.weight"],
                     T[f"{name}.noise_func.noise_func.0.bias"])[:, :, None, None]
    h = _block(T, f"{name}.block2", h, groups)
    r = F.conv2d(x, T[f"{name}.res_conv.weight"], T[f"{name}.res_conv.bias"]) if cin != cout else x
    return h + r


class UNetTorch:
    """Weights converted once; __call__(cond, x_t, noise_level) like oracle.unet.forward."""

    def __init__(self, P, arch):
        self.T = _t(P)
        self.arch = arch
        self.ev = torch.from_numpy(embedding_vector(arch["inner"]))

    @torch.no_grad()
    def __call__(self, cond, x_t, noise_level):
        T, arch = self.T, self.arch
        cond = torch.as_tensor(cond)
        x_t = torch.as_tensor(x_t)
        N = cond.shape[-1]
        idx = torch.from_numpy(frame_index(N, arch["seg"], arch["stride"]))
        x = torch.cat([cond[:, :, idx], x_t[:, :, idx]], dim=1)                          # :23-28, 244-247
        arg = torch.as_tensor(noise_level, dtype=torch.float32).reshape(-1, 1) * self.ev[None, :]
        enc = torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)                        # :57-68
        t = _swish(F.linear(enc, T["noise_level_mlp.1.weight"], T["noise_level_mlp.1.bias"]))
        t = _swish(F.linear(t, T["noise_level_mlp.3.weight"], T["noise_level_mlp.3.bias"]))
        G = arch["groups"]
        feats = []
        for kind, name, ci, co in arch["downs"]:                                         # :252-257
            if kind == "res":
                x = _resnet(T, name, x, t, G, ci, co)
            elif kind == "down":
                x = F.conv2d(x, T[f"{name}.conv.weight"], T[f"{name}.conv.bias"], stride=2, padding=1)
            else:
                x = F.conv2d(x, T[f"{name}.weight"], T[f"{name}.bias"], padding=1)
            feats.append(x)
        for kind, name, ci, co in arch["mid"]:                                           # :258-259
            x = _resnet(T, name, x, t, G, ci, co)
        for kind, name, ci, co in arch["ups"]:                                           # :261-265
            if kind == "res":
                x = _resnet(T, name, torch.cat([x, feats.pop()], dim=1), t, G, ci, co)
            else:
                x = F.interpolate(x, scale_factor=2, mode="nearest")
                x = F.conv2d(x, T[f"{name}.conv.weight"], T[f"{name}.conv.bias"], padding=1)
        y = _block(T, "final_conv", x, G)                                                # :267
        B, C, nf, W = y.shape                                                            # overlapAdd :30-41
        S = arch["stride"]
        out = torch.zeros((B, C, N), dtype=y.dtype)
        for k in range(W // S):        # frames f write [64 f + 64 k, +64): chunk k of every frame at once
            seg = y[:, :, :, k * S:(k + 1) * S].reshape(B, C, nf * S)
            out[:, :, k * S:k * S + nf * S] += seg
        return out.numpy()
