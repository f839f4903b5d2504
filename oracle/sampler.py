"""ORACLE (test infrastructure only) — reverse-diffusion sampler and transitions.

Restates, in fp32 with the reference's operation order:
  get_x_T              model/diffusion.py:281-300
  get_x_T_conditional  model/diffusion.py:302-320
  p_transition         model/diffusion.py:177-190
  p_transition_sr3     model/diffusion.py:164-175
  p_transition_supportive   model/diffusion.py:192-209
  p_transition_conditional  model/diffusion.py:211-223
  SDDM.infer (continuous=False)  model/model.py:50-124 (loop 106-122)
  SDDM_spectrogram.infer         model/model.py:212-257

Noise: ``oracle.philox.normal(seed, draw, shape, row_offset)`` with draw 0 for
x_T and draw t for the transition at step t (t > 1).
"""
import numpy as np

from . import philox

f32 = np.float32
MODES = ("original", "condition_in", "sr3", "supportive", "conditional")


def get_x_T(tab, cond, noise):
    T = len(tab["betas"]) - 1
    s = tab["sqrt_alpha_bar"][T]
    return (s * cond + np.sqrt(f32(1.0) - s * s) * noise).astype(np.float32)


def get_x_T_conditional(tab, cond, noise):
    T = len(tab["betas"]) - 1
    return (tab["sqrt_alpha_bar"][T] * cond + tab["sqrt_delta"][T] * noise).astype(np.float32)


def transition(mode, tab, x_t, t, eps, cond=None, noise=None):
    """One p_transition* step; ``noise`` used only when t > 1."""
    with np.errstate(invalid="ignore"):
        if mode in ("original", "condition_in"):
            x = (x_t - tab["predicted_noise_coeff"][t] * eps) / np.sqrt(tab["alphas"][t])
            if t > 1:
                x = x + tab["sigma"][t] * noise
        elif mode == "sr3":
            x = (x_t - tab["predicted_noise_coeff"][t] * eps) / np.sqrt(tab["alphas"][t])
            if t > 1:
                x = x + np.sqrt(tab["betas"][t]) * noise
        elif mode == "supportive":
            g = tab["supportive_gamma"][t]
            mu = x_t - tab["predicted_noise_coeff"][t] * eps
            x = ((f32(1.0) - g) * mu + g * cond) / np.sqrt(tab["alphas"][t])
            if t > 1:
                x = x + max(f32(0.0), tab["supportive_sigma_hat"][t]) * noise
        elif mode == "conditional":
            x = tab["c_xt"][t] * x_t + tab["c_yt"][t] * cond - tab["c_epst"][t] * eps
            if t > 1:
                x = x + tab["sqrt_delta_estimated"][t] * noise
        else:
            raise NotImplementedError(mode)
    return np.clip(x.astype(np.float32), f32(-1.0), f32(1.0))


def initial_state(mode, tab, cond, seed, row_offset=0, z=None):
    """x_T per SDDM.infer (model/model.py:57-68); z = the x_T draw (default: Philox draw 0)."""
    if mode == "supportive":
        return cond.astype(np.float32).copy()
    if z is None:
        z = philox.normal(seed, 0, cond.shape, row_offset)
    if mode == "conditional":
        return get_x_T_conditional(tab, cond, z)
    if mode == "condition_in":
        return get_x_T(tab, cond, z)
    return z


def infer(network, tab, cond, mode="condition_in", noise_condition="sqrt_alpha_bar", seed=7,
          row_offset=0, record=None, noise=None):
    """SDDM.infer (model/model.py:50-124): ``network(cond, x_t, noise_level[B]) -> eps``.
    noise: optional [T + 1, *cond.shape] draws (slot 0 = x_T, slot t = step t) in place of Philox."""
    T = len(tab["betas"]) - 1
    B = cond.shape[0]
    x = initial_state(mode, tab, cond, seed, row_offset, None if noise is None else noise[0])
    if record is not None:
        record.append(x.copy())
    for t in range(T, 0, -1):
        if noise_condition == "sqrt_alpha_bar":
            nl = np.full(B, tab["sqrt_alpha_bar"][t], dtype=np.float32)
        else:
            nl = np.full(B, float(t), dtype=np.float32)
        eps = network(cond, x, nl)
        z = (philox.normal(seed, t, x.shape, row_offset) if noise is None else noise[t]) if t > 1 else None
        x = transition(mode, tab, x, t, eps, cond, z)
        if record is not None:
            record.append(x.copy())
    return x


def infer_spectrogram(network, tab, spec, hop_samples, noise_condition="sqrt_alpha_bar", seed=7,
                      row_offset=0, noise=None):
    """SDDM_spectrogram.infer (model/model.py:212-257): x_T = randn(B,1,hop*F); noise as infer."""
    T = len(tab["betas"]) - 1
    B = spec.shape[0]
    shape = (B, 1, hop_samples * spec.shape[-1])
    x = philox.normal(seed, 0, shape, row_offset) if noise is None else noise[0].astype(np.float32)
    for t in range(T, 0, -1):
        if noise_condition == "sqrt_alpha_bar":
            nl = np.full(B, tab["sqrt_alpha_bar"][t], dtype=np.float32)
        else:
            nl = np.full(B, float(t), dtype=np.float32)
        eps = network(spec, x, nl)
        z = (philox.normal(seed, t, x.shape, row_offset) if noise is None else noise[t]) if t > 1 else None
        x = transition("original", tab, x, t, eps, None, z)
    return x


def q_stochastic(tab, x0, noise, t, r=None):
    """GaussianDiffusion.q_stochastic (diffusion.py:225-251) for given draws t [B] (int) and
    r [B] (uniform; None = t_is_integer).  Returns x_t, s [B], level [B]."""
    f32 = np.float32
    sab = tab["sqrt_alpha_bar"].astype(np.float32)
    if r is None:
        s = sab[t]
        level = t.astype(np.int64)
    else:
        la, lb = sab[t - 1], sab[t]
        s = (la + (r.astype(np.float32) * (lb - la)).astype(f32)).astype(f32)
        level = (t.astype(np.float32) + r.astype(np.float32)).astype(f32)
    sh = (-1,) + (1,) * (x0.ndim - 1)
    sv = s.reshape(sh)
    x_t = ((sv * x0).astype(f32) + (np.sqrt((f32(1.0) - (sv * sv).astype(f32)).astype(f32)) * noise).astype(f32))
    return x_t.astype(f32), s, level


def q_stochastic_conditional(tab, x0, y, noise, t):
    """GaussianDiffusion.q_stochastic_conditional (diffusion.py:253-279) for given t [B]."""
    f32 = np.float32
    sh = (-1,) + (1,) * (x0.ndim - 1)
    sab = tab["sqrt_alpha_bar"].astype(f32)[t].reshape(sh)
    g = (tab["sqrt_delta"].astype(f32)[t].reshape(sh) * noise).astype(f32)
    c = ((tab["m"].astype(f32)[t].reshape(sh) * sab).astype(f32) * (y - x0).astype(f32)).astype(f32)
    x_t = (((sab * x0).astype(f32) + c).astype(f32) + g).astype(f32)
    inv = (f32(1.0) / np.sqrt((f32(1.0) - tab["alpha_bar"].astype(f32)[t]).astype(f32))).astype(f32).reshape(sh)
    comb = (inv * (c + g).astype(f32)).astype(f32)
    return x_t, comb, sab.reshape(-1)
