"""GPU: forward-process noising (GaussianDiffusion.q_stochastic / q_stochastic_conditional,
reference diffusion.py:225-279) through the facade and sddm_q_sample, against reference goldens."""
import numpy as np
import pytest
import torch

from _helpers import golden, parse_sched_key

pytestmark = pytest.mark.gpu


def _draws(T, B, seed, integer=False, cond=False):
    torch.manual_seed(seed)                       # the reference's CPU-generator draws
    if cond:
        return torch.randint(1, T + 1, (B, 1, 1)), None
    t = torch.randint(1, T + 1, [B])
    return t, (None if integer else torch.rand(B))


@pytest.mark.parametrize("sk", ["linear_50_1e-06_0.001", "linear_200_0.0001_0.02"])
def test_q_stochastic_matches_reference(torch_cuda, sk):
    import model.diffusion as D
    z = golden("q_sample.npz")
    T = parse_sched_key(sk)[1]
    d = D.GaussianDiffusion(*parse_sched_key(sk), device="cuda")
    k = f"q/{sk}"
    x0, y, noise = (torch.from_numpy(z[f"{k}/{n}"]).cuda() for n in ("x0", "y", "noise"))
    for name, integer in (("float", False), ("int", True)):
        t, r = _draws(T, x0.shape[0], 5, integer)
        x_t, s, lvl = d.q_stochastic(x0, noise, t_is_integer=integer, t=t, random_step=r)
        assert x_t.shape == x0.shape and s.shape == (x0.shape[0], 1, 1) and lvl.shape == (x0.shape[0], 1, 1)
        assert np.abs(x_t.cpu().numpy() - z[f"{k}/{name}/x_t"]).max() <= 1e-6
        assert np.array_equal(s.cpu().numpy(), z[f"{k}/{name}/s"])
        assert np.array_equal(lvl.cpu().numpy(), z[f"{k}/{name}/level"])
        assert lvl.dtype == (torch.int64 if integer else torch.float32)
    t, _ = _draws(T, x0.shape[0], 6, cond=True)
    x_t, comb, s = d.q_stochastic_conditional(x0, y, noise, t=t)
    ref = z[f"{k}/cond/x_t"]
    ok = np.isfinite(ref)
    assert np.abs(x_t.cpu().numpy() - ref)[ok].max() <= 1e-6
    assert np.abs(comb.cpu().numpy() - z[f"{k}/cond/combined"])[ok].max() <= 1e-5
    assert np.array_equal(s.cpu().numpy(), z[f"{k}/cond/s"])


def test_q_stochastic_draws_like_reference_and_rejects_bad_t(torch_cuda):
    import model.diffusion as D
    d = D.GaussianDiffusion("linear", 100, 1e-4, 0.02, device="cuda")
    x0 = torch.rand(3, 1, 257, device="cuda")
    x_t, s, lvl = d.q_stochastic(x0, torch.randn_like(x0))
    assert torch.isfinite(x_t).all() and ((lvl >= 1) & (lvl < 101)).all()
    with pytest.raises(IndexError):
        d.q_stochastic(x0, torch.randn_like(x0), t=torch.tensor([0, 1, 2]))
