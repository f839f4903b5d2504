"""Sampler facade: SDDM (reference model/model.py:7-124) and SDDM_spectrogram (:206-257).

``SDDM.infer(condition)`` is the north-star hot path.  It hands the condition, the weights and
the schedule tables to libsddm_hip, which runs all T reverse steps (noise-level embedding,
UNetModified2 forward, p_transition with Philox noise) as HIP kernels on the caller's stream and
returns x_0.  Extra keyword arguments (all optional, defaults keep the reference behaviour):

  seed        noise-stream seed; default draws one from torch's CPU generator
  row_offset  global index of this batch's first row (multi-GPU sharding: rows keep the
              same noise whatever rank samples them)
  compute_dtype (constructor / attribute): 'float32' (parity, default), 'bfloat16', 'float16'
"""
import os

import torch
from torch import nn

import sddm_hip
from .diffusion import GaussianDiffusion, _seed_from_torch

_TUNING = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "conv_tuning.json")
_P_TRANSITIONS = ("original", "supportive", "sr3", "conditional", "condition_in")


class SDDM(nn.Module):
    def __init__(self, diffusion: GaussianDiffusion, noise_estimate_model: nn.Module,
                 noise_condition="sqrt_alpha_bar", p_transition="original", q_transition="original",
                 compute_dtype="float32"):
        super().__init__()
        self.diffusion = diffusion
        self.noise_estimate_model = noise_estimate_model
        self.num_timesteps = self.diffusion.num_timesteps
        self.noise_condition = noise_condition
        self.p_transition = p_transition
        self.q_transition = q_transition
        if noise_condition not in ("sqrt_alpha_bar", "time_step"):          # model.py:17-26
            raise NotImplementedError
        if p_transition not in _P_TRANSITIONS:
            raise NotImplementedError
        if q_transition not in ("original", "conditional"):
            raise NotImplementedError
        self.compute_dtype = compute_dtype
        self._ctx = None
        self._ctx_key = None

    def library_config(self):
        net = self.noise_estimate_model
        args = {"noise_condition": self.noise_condition, "p_transition": self.p_transition,
                "q_transition": self.q_transition}
        if hasattr(self, "hop_samples"):
            args = {"noise_condition": self.noise_condition, "hop_samples": self.hop_samples}
        return {"arch": {"type": type(self).__name__, "args": args},
                "diffusion": {"type": "GaussianDiffusion", "args": self.diffusion.schedule_args},
                "network": {"type": type(net).__name__, "args": net.config_args},
                "num_samples": getattr(net, "num_samples", -1)}

    def _context(self, device):
        sd = dict(self.state_dict())
        net = self.noise_estimate_model
        if hasattr(net, "library_params"):       # plain attributes the library needs (DiffWave)
            for k, v in net.library_params().items():
                sd.setdefault("noise_estimate_model." + k, v)
        key = (device.index or 0, self.compute_dtype) + tuple((k, v.data_ptr(), v._version) for k, v in sd.items())
        if self._ctx is None or self._ctx_key != key:
            ctx = sddm_hip.Context(self.library_config(), device.index or 0, self.compute_dtype)
            ctx.load_state_dict(sd)
            if os.path.exists(_TUNING) and not os.environ.get("SDDM_NO_TUNING"):   # measured per-layer kernels
                with open(_TUNING) as f:
                    ctx.set_conv_tuning(f.read())
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    def forward(self, target, condition):
        raise NotImplementedError("SDDM.forward is the training step (model.py:29-48), outside the sampling hot path")

    @torch.no_grad()
    def infer(self, condition, continuous=False, seed=None, row_offset=0):
        """Reverse diffusion x_T -> x_0 (model.py:50-124).  condition: [B, 1, N] on the HIP device."""
        if not condition.is_cuda:
            raise RuntimeError("SDDM.infer runs on the HIP device; move the condition to cuda")
        cond = condition.contiguous().float()
        ctx = self._context(cond.device)
        seed = _seed_from_torch() if seed is None else int(seed)
        out = torch.empty_like(cond)
        if not continuous:
            ctx.sample(cond, out, seed, row_offset)
            return out
        assert cond.shape[0] == 1, "Batch size must be 1 to do continuous sampling"   # model.py:80
        inter = 1 | (self.num_timesteps // 100)
        nrec = self.num_timesteps // inter
        record = torch.empty((max(nrec, 1),) + tuple(cond.shape), dtype=torch.float32, device=cond.device)
        ctx.sample_continuous(cond, out, record, inter, seed, row_offset)
        return [condition] + [record[i] for i in range(nrec)]


class SDDM_spectrogram(SDDM):
    """Spectrogram-conditioned sampler for DiffWave / WaveGrad (model.py:206-257)."""

    def __init__(self, diffusion: GaussianDiffusion, noise_estimate_model: nn.Module, hop_samples: int,
                 noise_condition="sqrt_alpha_bar", compute_dtype="float32"):
        super().__init__(diffusion, noise_estimate_model, noise_condition, compute_dtype=compute_dtype)
        self.hop_samples = hop_samples

    @torch.no_grad()
    def infer(self, condition, continuous=False, seed=None, row_offset=0):
        """Reverse diffusion from x_T = randn(B, 1, hop * F) (model.py:212-257).
        condition: spectrogram [B, bins, F] on the HIP device -> [B, 1, hop * F]."""
        if not condition.is_cuda:
            raise RuntimeError("SDDM_spectrogram.infer runs on the HIP device; move the condition to cuda")
        spec = condition.contiguous().float()
        ctx = self._context(spec.device)
        seed = _seed_from_torch() if seed is None else int(seed)
        B = spec.shape[0]
        out = torch.empty((B, 1, self.hop_samples * spec.shape[-1]), dtype=torch.float32, device=spec.device)
        if not continuous:
            ctx.sample(spec, out, seed, row_offset)
            return out
        assert B == 1, "Batch size must be 1 to do continuous sampling"             # model.py:224
        inter = 1 | (self.num_timesteps // 100)
        nrec = self.num_timesteps // inter
        record = torch.empty((max(nrec, 1),) + tuple(out.shape), dtype=torch.float32, device=spec.device)
        ctx.sample_continuous(spec, out, record, inter, seed, row_offset)
        return [condition] + [record[i] for i in range(nrec)]
