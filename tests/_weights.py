"""Deterministic test weights (test infrastructure).

The reference ships no checkpoint, so parity runs use
build-defined weights that depend only on (seed, parameter name, shape):

  conv / linear weight (ndim >= 2):  U(-1/sqrt(fan_in), 1/sqrt(fan_in))   (PyTorch's default bound)
  conv / linear bias:                same bound as its sibling weight
  GroupNorm weight (1-D .weight):    U(0.5, 1.5)
  GroupNorm bias (1-D .bias next to a 1-D .weight): U(-0.2, 0.2)

Element values come from the Philox stream of ``oracle.philox`` keyed by
(seed, crc32(name)), so the golden generator (which builds the reference
modules) and the tests (which build this package's modules) produce identical
tensors without storing 21 MB of weights.
"""
import zlib

import numpy as np

from oracle.philox import uniform_from_index


def _u(seed, name, n):
    return uniform_from_index(seed, zlib.crc32(name.encode()), np.arange(n, dtype=np.uint64))


def make_params(shapes, seed=0):
    """shapes: dict name -> tuple.  Returns dict name -> float32 array."""
    out = {}
    for name, shape in shapes.items():
        shape = tuple(int(s) for s in shape)
        n = int(np.prod(shape)) if shape else 1
        u = _u(seed, name, n)
        base = name.rsplit(".", 1)[0]
        wshape = shapes.get(base + ".weight")
        if name.endswith(".weight") and len(shape) >= 2:
            b = 1.0 / np.sqrt(np.prod(shape[1:]))
            v = (2 * u - 1) * b
        elif name.endswith(".weight"):
            v = 0.5 + u
        elif name.endswith(".bias") and wshape is not None and len(wshape) >= 2:
            b = 1.0 / np.sqrt(np.prod(wshape[1:]))
            v = (2 * u - 1) * b
        elif name.endswith(".bias"):
            v = (2 * u - 1) * 0.2
        else:
            v = (2 * u - 1) * 0.1
        out[name] = v.astype(np.float32).reshape(shape)
    return out


def unet_shapes(arch):
    """Parameter shapes of UNetModified2 (reference key names, no prefix)."""
    inner = arch["inner"]
    s = {"noise_level_mlp.1.weight": (inner * 4, inner), "noise_level_mlp.1.bias": (inner * 4,),
         "noise_level_mlp.3.weight": (inner, inner * 4), "noise_level_mlp.3.bias": (inner,)}

    def res(name, ci, co):
        s[f"{name}.noise_func.noise_func.0.weight"] = (co, inner)
        s[f"{name}.noise_func.noise_func.0.bias"] = (co,)
        s[f"{name}.block1.block.0.weight"] = (ci,)
        s[f"{name}.block1.block.0.bias"] = (ci,)
        s[f"{name}.block1.block.3.weight"] = (co, ci, 3, 3)
        s[f"{name}.block1.block.3.bias"] = (co,)
        s[f"{name}.block2.block.0.weight"] = (co,)
        s[f"{name}.block2.block.0.bias"] = (co,)
        s[f"{name}.block2.block.3.weight"] = (co, co, 3, 3)
        s[f"{name}.block2.block.3.bias"] = (co,)
        if ci != co:
            s[f"{name}.res_conv.weight"] = (co, ci, 1, 1)
            s[f"{name}.res_conv.bias"] = (co,)

    for kind, name, ci, co in arch["downs"] + arch["mid"] + arch["ups"]:
        if kind == "res":
            res(name, ci, co)
        elif kind in ("down", "up"):
            s[f"{name}.conv.weight"] = (co, ci, 3, 3)
            s[f"{name}.conv.bias"] = (co,)
        else:
            s[f"{name}.weight"] = (co, ci, 3, 3)
            s[f"{name}.bias"] = (co,)
    _, name, ci, co = arch["final"]
    s[f"{name}.block.0.weight"] = (ci,)
    s[f"{name}.block.0.bias"] = (ci,)
    s[f"{name}.block.3.weight"] = (co, ci, 3, 3)
    s[f"{name}.block.3.bias"] = (co,)
    return s
