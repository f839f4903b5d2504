"""ORACLE (test infrastructure only) — GaussianDiffusion schedule tables.

Restates model/diffusion.py:49-161 (``GaussianDiffusion.__init__``,
``calculate_p_coeffs``, ``calculate_coeffs_conditional``) in float32 with the
exact rounding torch uses on CPU:

* ``torch.linspace`` (diffusion.py:67,71): step = (end - start) / (n - 1) in fp32;
  element i < n//2 is fmaf(step, i, start), the rest fmaf(-step, n-1-i, end)
  (SURVEY.md §8a "Numerical facts");
* ``torch.cumprod`` (diffusion.py:69,73): float64 running product rounded to
  fp32 per element;
* every other op is a single fp32 operation (numpy float32 arithmetic is IEEE
  per-op rounded), ``x ** 0.5`` is sqrt and ``x ** 2`` is x * x as in ATen.
"""
from fractions import Fraction
import math
import numpy as np

f32 = np.float32
BUFFER_NAMES = ("betas", "alphas", "alpha_bar", "sqrt_alpha_bar", "predicted_noise_coeff",
                "sigma", "supportive_gamma", "supportive_sigma_hat", "m", "sqrt_delta",
                "c_xt", "c_yt", "c_epst", "sqrt_delta_estimated")


def _round_f32(fr):
    """Correctly rounded (nearest-even) fp32 of an exact Fraction."""
    x = np.float32(float(fr))
    best = None
    for cand in (np.nextafter(x, np.float32(-np.inf)), x, np.nextafter(x, np.float32(np.inf))):
        if not np.isfinite(cand):
            continue
        err = abs(Fraction(float(cand)) - fr)
        key = (err, int(np.frombuffer(np.float32(cand).tobytes(), np.uint32)[0]) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return np.float32(best[1])


def fmaf(a, b, c):
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def linspace_f32(start, end, n):
    """torch.linspace(start, end, n, dtype=float32) on CPU (diffusion.py:67)."""
    s, e = f32(start), f32(end)
    out = np.empty(n, dtype=np.float32)
    if n == 1:
        out[0] = s
        return out
    step = f32(e - s) / f32(n - 1)
    half = n // 2
    for i in range(n):
        out[i] = fmaf(step, i, s) if i < half else fmaf(-step, n - 1 - i, e)
    return out


def cumprod_f32(a):
    """torch.cumprod(fp32) on CPU: float64 accumulator, rounded per element."""
    acc = 1.0
    out = np.empty_like(a, dtype=np.float32)
    for i, v in enumerate(a):
        acc *= float(v)
        out[i] = f32(acc)
    return out


def make_tables(schedule="linear", n_timestep=1000, linear_start=1e-4, linear_end=2e-2):
    """All 14 registered buffers of GaussianDiffusion (diffusion.py:50-161), each [T+1] fp32."""
    T = int(n_timestep)
    one = f32(1.0)
    with np.errstate(invalid="ignore", divide="ignore"):
        betas = np.zeros(T + 1, dtype=np.float32)
        if schedule == "linear":                                   # diffusion.py:66-69
            betas[1:] = linspace_f32(linear_start, linear_end, T)
            alphas = one - betas
            alpha_bar = cumprod_f32(alphas)
        elif schedule == "quad":                                   # diffusion.py:70-73
            lin = linspace_f32(linear_start ** 0.5, linear_end ** 0.5, T)
            betas[1:] = lin * lin
            alphas = one - betas
            alpha_bar = cumprod_f32(alphas)
        elif schedule == "cosine":                                 # diffusion.py:74-82
            ts = np.arange(T + 1, dtype=np.float32) / f32(T) + f32(0.008)
            f = ts / f32(1 + 0.008) * f32(math.pi / 2)
            f = np.cos(f.astype(np.float64)).astype(np.float32)
            f = f * f
            alpha_bar = f / f[0]
            betas[1:] = one - alpha_bar[1:] / alpha_bar[:-1]
            betas = np.minimum(betas, f32(0.999))
            alphas = one - betas
        else:
            raise NotImplementedError(schedule)
        sqrt_alpha_bar = np.sqrt(alpha_bar)

        # calculate_p_coeffs (diffusion.py:98-117)
        sigma = np.zeros_like(betas)
        sigma[1:] = np.sqrt((one - alpha_bar[:-1]) / (one - alpha_bar[1:]) * betas[1:])
        pnc = np.zeros_like(betas)
        pnc[1:] = betas[1:] / np.sqrt(one - alpha_bar[1:])
        sg = np.zeros_like(betas)
        sg[1] = f32(0.2)
        sg[2:] = sigma[2:]
        ssh = np.zeros_like(betas)
        ssh[1:] = sigma[1:] - sg[1:] / np.sqrt(alphas[1:])

        # calculate_coeffs_conditional (diffusion.py:119-161)
        m = np.sqrt((one - alpha_bar) / sqrt_alpha_bar)
        delta = (one - alpha_bar) - (m * m) * alpha_bar
        sqrt_delta = np.sqrt(delta)
        omr = (one - m[1:]) / (one - m[:-1])
        atd = alphas[1:] * delta[:-1]
        dtg = delta[1:] - (omr * omr) * atd
        sqa = np.sqrt(alphas[1:])
        c_xt = np.zeros_like(betas)
        c_xt[1:] = omr * delta[:-1] / delta[1:] * sqa + (one - m[:-1]) * (dtg / delta[1:]) * (one / sqa)
        c_yt = np.zeros_like(betas)
        c_yt[1:] = (m[:-1] * delta[1:] - m[1:] * omr * atd) * sqrt_alpha_bar[:-1] / delta[1:]
        c_epst = np.zeros_like(betas)
        c_epst[1:] = (one - m[:-1]) * dtg / delta[1:] * np.sqrt(one - alpha_bar[1:]) / sqa
        de = np.zeros_like(betas)
        de[1:] = dtg * delta[:-1] / delta[1:]
        sde = np.sqrt(de)
    return dict(zip(BUFFER_NAMES, (betas, alphas, alpha_bar, sqrt_alpha_bar, pnc, sigma, sg, ssh,
                                   m, sqrt_delta, c_xt, c_yt, c_epst, sde)))
