"""Sampler facade: SDDM (reference model/model.py:7-124) and SDDM_spectrogram (:206-257).

``SDDM.infer(condition)`` is the north-star hot path.  It hands the condition, the weights and
the schedule tables to libsddm_hip, which runs all T reverse steps (noise-level embedding,
UNetModified2 forward, p_transition with Philox noise) as HIP kernels on the caller's stream and
returns x_0.  Extra keyword arguments (all optional, defaults keep the reference behaviour):

  seed        noise-stream seed; default draws one from torch's CPU generator
  row_offset  global index of this batch's first row (multi-GPU sharding: rows keep the
              same noise whatever rank samples them)
  noise       caller-supplied Gaussian draws [T + 1, *x_T.shape] (SURVEY §8(b) noise_mode 1) in place
              of the device Philox stream; reference_noise() draws them with torch exactly as the
              reference's infer does, so the output matches the reference run from the same torch seed
  compute_dtype (constructor / attribute): 'float32' (parity, default), 'bfloat16', 'float16'
  lane_rows   (attribute): rows per lane of the UNet plan (library default 16; 64 for per-GPU
              batches of 64+ rows, e.g. config #5)
"""
import os

import torch
from torch import nn

import sddm_hip
from .diffusion import GaussianDiffusion, _seed_from_torch

_TUNING = os.environ.get("SDDM_TUNING_FILE") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "conv_tuning.json")
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
        self.lane_rows = None
        self._ctx = None
        self._ctx_key = None

    def library_config(self):
        net = self.noise_estimate_model
        args = {"noise_condition": self.noise_condition, "p_transition": self.p_transition,
                "q_transition": self.q_transition}
        if hasattr(self, "hop_samples"):
            args = {"noise_condition": self.noise_condition, "hop_samples": self.hop_samples}
        cfg = {"arch": {"type": type(self).__name__, "args": args},
               "diffusion": {"type": "GaussianDiffusion", "args": self.diffusion.schedule_args},
               "network": {"type": type(net).__name__, "args": net.config_args},
               "num_samples": getattr(net, "num_samples", -1)}
        if getattr(self, "lane_rows", None):
            cfg["lane_rows"] = int(self.lane_rows)
        return cfg

    def _context(self, device):
        sd = dict(self.state_dict())
        net = self.noise_estimate_model
        if hasattr(net, "library_params"):       # plain attributes the library needs (DiffWave)
            for k, v in net.library_params().items():
                sd.setdefault("noise_estimate_model." + k, v)
        key = (device.index or 0, self.compute_dtype, getattr(self, "lane_rows", None)) + tuple((k, v.data_ptr(), v._version) for k, v in sd.items())
        if self._ctx is None or self._ctx_key != key:
            ctx = sddm_hip.Context(self.library_config(), device.index or 0, self.compute_dtype)
            ctx.load_state_dict(sd)
            if os.path.exists(_TUNING) and not os.environ.get("SDDM_NO_TUNING"):   # measured per-layer kernels
                with open(_TUNING) as f:
                    ctx.set_conv_tuning(f.read())
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    def forward(self, target, condition, noise=None, t=None, random_step=None):
        """Training-step forward (model.py:29-48): q-sample x_t from the target, estimate its noise.
        Returns (predicted, noise) like the reference.  Both pieces run on HIP (sddm_q_sample, then
        the network forward); the draws (randn_like / randint / rand on the target's device) are the
        reference's unless given.  Evaluation only: the HIP path has no backward, so a call that
        would build an autograd graph (grad mode on, parameters requiring grad: the reference's
        Trainer._train_epoch, trainer.py:64-73) raises instead of returning tensors without history."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError(
                "SDDM.forward on HIP has no backward (no training step): call it under torch.no_grad() "
                "or with the parameters' requires_grad off")
        with torch.no_grad():
            return self._forward_eval(target, condition, noise, t, random_step)

    def _forward_eval(self, target, condition, noise, t, random_step):
        if not target.is_cuda:
            raise RuntimeError("SDDM.forward runs on the HIP device; move the tensors to cuda")
        if noise is None:
            noise = torch.randn_like(target, device=target.device)
        net = self.noise_estimate_model
        if self.q_transition == "original":
            x_t, noise_level, steps = self.diffusion.q_stochastic(target, noise, t=t, random_step=random_step)
            level = noise_level if self.noise_condition == "sqrt_alpha_bar" else steps
            predicted = net(condition, x_t, level)
        else:
            x_t, noise, noise_level = self.diffusion.q_stochastic_conditional(target, condition, noise, t=t)
            predicted = net(condition, x_t, noise_level)
        return predicted, noise

    @torch.no_grad()
    def infer(self, condition, continuous=False, seed=None, row_offset=0, noise=None):
        """Reverse diffusion x_T -> x_0 (model.py:50-124).  condition: [B, 1, N] on the HIP device."""
        if not condition.is_cuda:
            raise RuntimeError("SDDM.infer runs on the HIP device; move the condition to cuda")
        cond = condition.contiguous().float()
        ctx = self._context(cond.device)
        out = torch.empty_like(cond)
        if noise is not None:
            if continuous:
                raise NotImplementedError("caller-supplied noise with continuous sampling")
            ctx.sample_noise(cond, out, _noise_buffer(noise, self.num_timesteps, out))
            return out
        seed = _seed_from_torch() if seed is None else int(seed)
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
    def infer(self, condition, continuous=False, seed=None, row_offset=0, noise=None):
        """Reverse diffusion from x_T = randn(B, 1, hop * F) (model.py:212-257).
        condition: spectrogram [B, bins, F] on the HIP device -> [B, 1, hop * F]."""
        if not condition.is_cuda:
            raise RuntimeError("SDDM_spectrogram.infer runs on the HIP device; move the condition to cuda")
        spec = condition.contiguous().float()
        bins = getattr(self.noise_estimate_model, "freq_bins", None)
        if bins is not None and (spec.dim() != 3 or spec.shape[1] != bins):
            raise RuntimeError(f"{type(self.noise_estimate_model).__name__} expects a spectrogram condition "
                               f"[B, {bins}, frames], got {tuple(spec.shape)}")
        ctx = self._context(spec.device)
        B = spec.shape[0]
        out = torch.empty((B, 1, self.hop_samples * spec.shape[-1]), dtype=torch.float32, device=spec.device)
        if noise is not None:
            if continuous:
                raise NotImplementedError("caller-supplied noise with continuous sampling")
            ctx.sample_noise(spec, out, _noise_buffer(noise, self.num_timesteps, out))
            return out
        seed = _seed_from_torch() if seed is None else int(seed)
        if not continuous:
            ctx.sample(spec, out, seed, row_offset)
            return out
        assert B == 1, "Batch size must be 1 to do continuous sampling"             # model.py:224
        inter = 1 | (self.num_timesteps // 100)
        nrec = self.num_timesteps // inter
        record = torch.empty((max(nrec, 1),) + tuple(out.shape), dtype=torch.float32, device=spec.device)
        ctx.sample_continuous(spec, out, record, inter, seed, row_offset)
        return [condition] + [record[i] for i in range(nrec)]


def _noise_buffer(noise, T, out):
    """Caller noise as the contiguous fp32 [T + 1][B][N] device buffer of sddm_sample_noise."""
    n = torch.as_tensor(noise)
    if tuple(n.shape) != (T + 1,) + tuple(out.shape):
        raise ValueError(f"noise must be [T + 1 = {T + 1}, {tuple(out.shape)}], got {tuple(n.shape)}")
    return n.to(device=out.device, dtype=torch.float32).contiguous()


def reference_noise(model, condition, device=None, generator=None):
    """The standard-normal draws the reference's infer makes, in its order, as [T + 1, *x_T.shape]:
    slot 0 = x_T's draw (SDDM: get_x_T / get_x_T_conditional / randn_like, none for 'supportive',
    model.py:57-68; SDDM_spectrogram: torch.randn(B, 1, hop F), model.py:216), slot t = the
    p_transition* draw of step t for t = T .. 2 (diffusion.py:172,187,207,220).  Drawn with
    torch.randn on `device` (default: the condition's, as the reference) from `generator` (default:
    that device's default generator), so seeding torch as a reference run did reproduces its noise."""
    T = model.num_timesteps
    device = condition.device if device is None else torch.device(device)
    if hasattr(model, "hop_samples"):
        shape = (condition.shape[0], 1, model.hop_samples * condition.shape[-1])
    else:
        shape = tuple(condition.shape)
    out = torch.zeros((T + 1,) + shape, dtype=torch.float32)
    if hasattr(model, "hop_samples") or model.p_transition != "supportive":
        out[0] = torch.randn(shape, device=device, generator=generator).cpu()
    for t in range(T, 1, -1):
        out[t] = torch.randn(shape, device=device, generator=generator).cpu()
    return out


# ---------------------------------------------------------------------------------------------
# Multi-GPU sampling.  The reference's only multi-GPU path is DataParallel
# (infer.py:49-50), which cannot call .infer.  Here the batch rows are sharded across
# the ranks of a torch.distributed group (one process per GPU): contiguous row blocks, the batch
# padded to a multiple of the world size, every rank samples its block with row_offset = its
# first global row (the noise is keyed by global row, so the rows equal a single-GPU run bit for
# bit), then ONE all-gather of the outputs (RCCL over xGMI with the nccl backend).
# ---------------------------------------------------------------------------------------------
def _all_gather_rows(out, group):
    import torch.distributed as dist
    P = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":          # gloo gathers host tensors (CPU tests, shared-GPU tests)
        host = out.detach().cpu().contiguous()
        parts = [torch.empty_like(host) for _ in range(P)]
        dist.all_gather(parts, host, group=group)
        return torch.cat(parts).to(out.device)
    gathered = torch.empty((P * out.shape[0],) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
    dist.all_gather_into_tensor(gathered, out.contiguous(), group=group)
    return gathered


def sharded_infer(model, condition, seed=None, group=None):
    """model.infer over the ranks of `group`; every rank passes the same full `condition` [B, ...]
    and gets the full [B, 1, N] output.  Without an initialised process group this is model.infer."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return model.infer(condition, seed=seed)
    P, r = dist.get_world_size(group), dist.get_rank(group)
    if seed is None:                               # one seed for every rank (rank 0's generator)
        s = torch.tensor([_seed_from_torch() if r == 0 else 0], dtype=torch.int64)
        if dist.get_backend(group) != "gloo":
            s = s.to(condition.device)
        dist.broadcast(s, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        seed = int(s.item())
    B = condition.shape[0]
    per = -(-B // P)
    if per * P != B:                               # pad to a multiple of the world size (§8e)
        pad = torch.zeros((per * P - B,) + tuple(condition.shape[1:]), dtype=condition.dtype, device=condition.device)
        condition = torch.cat([condition, pad])
    mine = condition[r * per:(r + 1) * per].contiguous()
    out = model.infer(mine, seed=seed, row_offset=r * per)
    return _all_gather_rows(out, group)[:B]


# ---------------------------------------------------------------------------------------------
# Building the sampler from a reference config (the plugin surface of parse_config.py:82-95).
# The spectrogram models need kwargs the reference's own scripts derive from the config
# (train_specmodel.py:21-49): freq_bins, num_timesteps and hop_samples.  config_diffwave.json
# names its bin count 'stft_bins'  and gives no arch hop_samples (Q6); both resolve
# from the config's 'spectrogram' section.
# ---------------------------------------------------------------------------------------------
_SPEC_NETS = ("DiffWave", "WaveGrad")


def spectrogram_kwargs(config, diffusion):
    """(network kwargs, arch kwargs) for init_obj of a spectrogram-conditioned model."""
    cfg = config.config if hasattr(config, "config") else config
    spec = cfg.get("spectrogram", {})
    if cfg.get("datatype", ".spec.npy") == ".mel.npy" or _dataset_datatype(cfg) == ".mel.npy":
        spec = cfg.get("mel_spectrogram", spec)
        bins = spec["n_mels"]
    else:
        bins = spec.get("freq_bins", spec.get("stft_bins", spec.get("window_length", 1024) // 2 + 1))
    net_kw = {"num_samples": cfg.get("num_samples", -1), "freq_bins": bins, "num_timesteps": diffusion.num_timesteps}
    arch_kw = {}
    if "hop_samples" not in cfg["arch"].get("args", {}):
        arch_kw["hop_samples"] = spec.get("hop_samples", 300 if cfg["network"]["type"] == "WaveGrad" else 256)
    return net_kw, arch_kw


def _dataset_datatype(cfg):
    """The spectrogram file type the config's datasets read (config_diffwave.json:44,51 put
    'datatype' under the dataset args, train_specmodel.py:21 reads a top-level one): the top-level
    key, else infer_dataset's, else tr_dataset's."""
    if "datatype" in cfg:
        return cfg["datatype"]
    for k in ("infer_dataset", "tr_dataset", "val_dataset"):
        dt = cfg.get(k, {}).get("args", {}).get("datatype")
        if dt:
            return dt
    return None


def build_from_config(config, module_diffusion, module_network, module_arch, device):
    """diffusion, network and arch objects exactly as the reference's scripts build them."""
    cfg = config.config if hasattr(config, "config") else config
    diffusion = config.init_obj("diffusion", module_diffusion, device=device)
    if cfg["network"]["type"] in _SPEC_NETS:
        net_kw, arch_kw = spectrogram_kwargs(config, diffusion)
        network = config.init_obj("network", module_network, **net_kw)
        model = config.init_obj("arch", module_arch, diffusion, network, **arch_kw)
    else:
        network = config.init_obj("network", module_network, num_samples=cfg["num_samples"])
        model = config.init_obj("arch", module_arch, diffusion, network)
    return diffusion, network, model
