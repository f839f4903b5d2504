"""GaussianDiffusion facade (reference model/diffusion.py:49-326).

Same constructor, same 14 registered buffers (so ``state_dict`` keys and values match and a
reference checkpoint loads unchanged), same transition methods.  The tables come from the
library's host schedule code (bit-exact linspace / cumprod rules); every transition runs as a
HIP kernel through the C ABI on CUDA tensors.  Sampling noise is the counter-based Philox stream
(draw t at step t, draw 0 for x_T); the seed is drawn from torch's CPU generator when not given,
so ``torch.manual_seed`` keeps controlling reproducibility as in the reference.
"""
import torch
from torch import nn

import sddm_hip


def _seed_from_torch():
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class GaussianDiffusion(nn.Module):
    def __init__(self, schedule="linear", n_timestep=1000, linear_start=1e-4, linear_end=2e-2, device="cuda"):
        super().__init__()
        self.num_timesteps = n_timestep
        self.device = device
        self.schedule_args = {"schedule": schedule, "n_timestep": int(n_timestep),
                              "linear_start": float(linear_start), "linear_end": float(linear_end)}
        tabs = sddm_hip.schedule(schedule, n_timestep, linear_start, linear_end)   # NotImplementedError
        dev = torch.device(device) if not (str(device).startswith("cuda") and not torch.cuda.is_available()) \
            else torch.device("cpu")
        for name in sddm_hip.TABLE_NAMES:                                            # diffusion.py:89-161
            self.register_buffer(name, torch.from_numpy(tabs[name].copy()).to(dev))
        self._ctx = None
        self._ctx_key = None

    # ---- library context holding only the tables (transitions / initial states) ----
    def _context(self, device):
        key = (device.index or 0,) + tuple((getattr(self, n).data_ptr(), getattr(self, n)._version)
                                           for n in sddm_hip.TABLE_NAMES)
        if self._ctx is None or self._ctx_key != key:
            ctx = sddm_hip.Context({"arch": {"type": "SDDM", "args": {}},
                                    "diffusion": {"type": "GaussianDiffusion", "args": self.schedule_args}},
                                   device.index or 0)
            for n in sddm_hip.TABLE_NAMES:
                ctx.load_param("diffusion." + n, getattr(self, n).detach().float().cpu().numpy())
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    def _transition(self, mode, x_t, t, predicted, condition=None, seed=None, row_offset=0):
        if not x_t.is_cuda:
            raise RuntimeError("GaussianDiffusion transitions run on the HIP device; move tensors to cuda")
        x_t = x_t.contiguous().float()
        out = torch.empty_like(x_t)
        self._context(x_t.device).transition(mode, x_t, predicted.contiguous().float(),
                                             None if condition is None else condition.contiguous().float(),
                                             int(t), out, _seed_from_torch() if seed is None else seed, row_offset)
        return out

    @torch.no_grad()
    def p_transition(self, x_t, t, predicted, seed=None, row_offset=0):
        """Ho et al. transition (diffusion.py:177-190)."""
        return self._transition(sddm_hip.TR_ORIGINAL, x_t, t, predicted, None, seed, row_offset)

    @torch.no_grad()
    def p_transition_sr3(self, x_t, t, predicted, seed=None, row_offset=0):
        """sr3 variance (diffusion.py:164-175)."""
        return self._transition(sddm_hip.TR_SR3, x_t, t, predicted, None, seed, row_offset)

    @torch.no_grad()
    def p_transition_supportive(self, x_t, t, predicted_noise, condition, seed=None, row_offset=0):
        """Lu et al. supportive transition (diffusion.py:192-209)."""
        return self._transition(sddm_hip.TR_SUPPORTIVE, x_t, t, predicted_noise, condition, seed, row_offset)

    @torch.no_grad()
    def p_transition_conditional(self, x_t, t, predicted_noise, condition, seed=None, row_offset=0):
        """Conditional transition (diffusion.py:211-223)."""
        return self._transition(sddm_hip.TR_CONDITIONAL, x_t, t, predicted_noise, condition, seed, row_offset)

    def _x_T(self, mode, condition, seed, row_offset):
        if not condition.is_cuda:
            raise RuntimeError("GaussianDiffusion.get_x_T runs on the HIP device; move tensors to cuda")
        c = condition.contiguous().float()
        out = torch.empty_like(c)
        self._context(c.device).initial_state(mode, c, out, _seed_from_torch() if seed is None else seed, row_offset)
        return out

    def get_x_T(self, condition, seed=None, row_offset=0):
        """sqrt(ab_T) * cond + sqrt(1 - ab_T) * eps (diffusion.py:281-300)."""
        return self._x_T(sddm_hip.TR_CONDITION_IN, condition, seed, row_offset)

    def get_x_T_conditional(self, condition, seed=None, row_offset=0):
        """sqrt(ab_T) * cond + sqrt(delta_T) * eps (diffusion.py:302-320)."""
        return self._x_T(sddm_hip.TR_CONDITIONAL, condition, seed, row_offset)

    def get_noise_level(self, t):
        """sqrt(alpha_bar[t]) (diffusion.py:322-326)."""
        return self.sqrt_alpha_bar[t]

    # ---- forward process (training-side q_sample, diffusion.py:225-279) on the HIP device ----
    def _q(self, mode, x_0, y, noise, t, r):
        if not x_0.is_cuda:
            raise RuntimeError("GaussianDiffusion.q_stochastic runs on the HIP device; move tensors to cuda")
        b = x_0.shape[0]
        x0 = x_0.contiguous().float()
        t_dev = t.reshape(-1).to(device=x0.device, dtype=torch.int64).contiguous()
        if t_dev.numel() != b or int(t_dev.min()) < 1 or int(t_dev.max()) > self.num_timesteps:
            raise IndexError("q_stochastic: t must hold one step in [1, num_timesteps] per batch row")
        r_dev = None if r is None else r.reshape(-1).to(device=x0.device, dtype=torch.float32).contiguous()
        x_t = torch.empty_like(x0)
        comb = torch.empty_like(x0) if mode == 1 else None
        s_out = torch.empty(b, dtype=torch.float32, device=x0.device)
        lvl = torch.empty(b, dtype=torch.float32, device=x0.device) if mode == 0 else None
        self._context(x0.device).q_sample(mode, x0, None if y is None else y.contiguous().float(),
                                          noise.contiguous().float(), t_dev, r_dev, x_t, comb, s_out, lvl)
        return x_t, comb, s_out, lvl, t_dev

    @torch.no_grad()
    def q_stochastic(self, x_0, noise, t_is_integer=False, t=None, random_step=None):
        """x_t = s x_0 + sqrt(1 - s^2) noise with s uniform between sqrt_alpha_bar[t-1] and
        sqrt_alpha_bar[t] (diffusion.py:225-251).  t / random_step are drawn like the reference
        (torch.randint / torch.rand on x_0's device) unless given."""
        b = x_0.shape[0]
        shape = (b,) + (1,) * (x_0.ndim - 1)
        if t is None:
            t = torch.randint(1, self.num_timesteps + 1, [b], device=x_0.device)
        if not t_is_integer and random_step is None:
            random_step = torch.rand(b, device=x_0.device)
        x_t, _, s, lvl, t_dev = self._q(0, x_0, None, noise, t, None if t_is_integer else random_step)
        level = t_dev.view(shape) if t_is_integer else lvl.view(shape)
        return x_t, s.view(shape), level

    @torch.no_grad()
    def q_stochastic_conditional(self, x_0, y, noise, t=None):
        """x_t = sab[t] x_0 + m[t] sab[t] (y - x_0) + sqrt_delta[t] noise and the combined noise
        (diffusion.py:253-279)."""
        b = x_0.shape[0]
        shape = (b,) + (1,) * (x_0.ndim - 1)
        if t is None:
            t = torch.randint(1, self.num_timesteps + 1, shape, device=x_0.device)
        x_t, comb, s, _, _ = self._q(1, x_0, y, noise, t, None)
        return x_t, comb, s.view(shape)
