"""Shared test helpers: fixtures, configs and deterministic weights (test infrastructure)."""
import copy
import os

import numpy as np

from oracle import schedule as osched
from oracle import unet as ounet
from _weights import make_params, unet_shapes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

UNET_NET = {"type": "UNetModified2",
            "args": {"in_channel": 2, "out_channel": 1, "inner_channel": 32, "norm_groups": 32,
                     "channel_mults": [1, 2, 3, 4, 5], "res_blocks": 1, "dropout": 0,
                     "segment_len": 128, "segment_stride": 64}}   # config_unet.json "network"


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def sched_key(s):
    return f"{s[0]}_{s[1]}_{s[2]:g}_{s[3]:g}"


def parse_sched_key(k):
    name, T, a, b = k.split("_")
    return name, int(T), float(a), float(b)


def tables_from_golden(key):
    S = golden("schedules.npz")
    return {k: S[f"sched/{key}/{k}"] for k in osched.BUFFER_NAMES}


def unet_config(num_samples, sched=("linear", 100, 1e-6, 1e-3), p_transition="condition_in"):
    return {"arch": {"type": "SDDM", "args": {"p_transition": p_transition, "q_transition": "original"}},
            "diffusion": {"type": "GaussianDiffusion",
                          "args": {"schedule": sched[0], "n_timestep": sched[1],
                                   "linear_start": sched[2], "linear_end": sched[3]}},
            "network": copy.deepcopy(UNET_NET), "num_samples": num_samples}


def unet_arch(num_samples):
    a = UNET_NET["args"]
    return ounet.architecture(num_samples, inner_channel=a["inner_channel"], norm_groups=a["norm_groups"],
                              channel_mults=tuple(a["channel_mults"]), res_blocks=a["res_blocks"],
                              segment_len=a["segment_len"], segment_stride=a["segment_stride"])


def unet_params(num_samples, seed=0):
    return make_params(unet_shapes(unet_arch(num_samples)), seed)


def rms(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)))


def diffwave_params(seed=0, bins=513):
    """Deterministic DiffWave weights with the reference key names (no module prefix)."""
    from oracle.diffwave import param_shapes
    return make_params(param_shapes(bins), seed)


def wavegrad_params(seed=0):
    """Deterministic WaveGrad weights with the reference key names (no module prefix)."""
    from oracle.wavegrad import param_shapes
    return make_params(param_shapes(), seed)
