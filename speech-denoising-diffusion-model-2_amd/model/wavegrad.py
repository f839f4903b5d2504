"""WaveGrad facade (reference model/wavegrad.py:9-179).

The module tree only *holds parameters*: class names, attribute names and shapes follow the
reference so that ``state_dict()`` / ``load_state_dict`` exchange reference checkpoints unchanged.
``forward`` never computes in torch: every convolution (DBlocks, FiLMs, UBlocks, first/last conv)
runs as a HIP kernel in libsddm_hip (csrc/wavegrad.hip).

Deviation: the reference's ``SDDM_spectrogram`` hands WaveGrad a [B,1,N] x_t, which
its Conv1d rejects (4-D input), and WaveGrad's squeezed [B,N] output would broadcast against x_t.
The library applies the adapter (audio = x_t[:, 0], noise level [B], eps -> [B,1,N]); this
``forward`` accepts audio as [B,N] (reference) or [B,1,N] and returns ``squeeze``d output like
the reference (wavegrad.py:179).
"""
from math import log as ln  # noqa: F401  (reference import surface)

import torch
from torch import nn

import sddm_hip
from .diffwave import check_spectrogram


class Conv1d(nn.Conv1d):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.reset_parameters()

    def reset_parameters(self):                                      # wavegrad.py:14-16
        nn.init.orthogonal_(self.weight)
        nn.init.zeros_(self.bias)


class PositionalEncoding(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim


class FiLM(nn.Module):
    def __init__(self, input_size, output_size):
        super().__init__()
        self.encoding = PositionalEncoding(input_size)
        self.input_conv = nn.Conv1d(input_size, input_size, 3, padding=1)
        self.output_conv = nn.Conv1d(input_size, output_size * 2, 3, padding=1)
        nn.init.xavier_uniform_(self.input_conv.weight)              # wavegrad.py:60-64
        nn.init.xavier_uniform_(self.output_conv.weight)
        nn.init.zeros_(self.input_conv.bias)
        nn.init.zeros_(self.output_conv.bias)


class UBlock(nn.Module):
    def __init__(self, input_size, hidden_size, factor, dilation):
        super().__init__()
        assert isinstance(dilation, (list, tuple))
        assert len(dilation) == 4
        self.factor = factor
        self.block1 = Conv1d(input_size, hidden_size, 1)
        self.block2 = nn.ModuleList([
            Conv1d(input_size, hidden_size, 3, dilation=dilation[0], padding=dilation[0]),
            Conv1d(hidden_size, hidden_size, 3, dilation=dilation[1], padding=dilation[1])])
        self.block3 = nn.ModuleList([
            Conv1d(hidden_size, hidden_size, 3, dilation=dilation[2], padding=dilation[2]),
            Conv1d(hidden_size, hidden_size, 3, dilation=dilation[3], padding=dilation[3])])


class DBlock(nn.Module):
    def __init__(self, input_size, hidden_size, factor):
        super().__init__()
        self.factor = factor
        self.residual_dense = Conv1d(input_size, hidden_size, 1)
        self.conv = nn.ModuleList([
            Conv1d(input_size, hidden_size, 3, dilation=1, padding=1),
            Conv1d(hidden_size, hidden_size, 3, dilation=2, padding=2),
            Conv1d(hidden_size, hidden_size, 3, dilation=4, padding=4)])


class WaveGrad(nn.Module):
    """wavegrad.py:140-179.  The reference constructor takes no arguments; the keyword arguments
    ConfigParser.init_obj adds (num_samples, freq_bins, num_timesteps) are accepted and ignored."""

    hop_samples = 300
    freq_bins = 128                      # first_conv = Conv1d(128, 768, 3) (wavegrad.py:164)

    def __init__(self, **unused):
        super().__init__()
        self.downsample = nn.ModuleList([
            Conv1d(1, 32, 5, padding=2),
            DBlock(32, 128, 2),
            DBlock(128, 128, 2),
            DBlock(128, 256, 3),
            DBlock(256, 512, 5)])
        self.film = nn.ModuleList([
            FiLM(32, 128),
            FiLM(128, 128),
            FiLM(128, 256),
            FiLM(256, 512),
            FiLM(512, 512)])
        self.upsample = nn.ModuleList([
            UBlock(768, 512, 5, [1, 2, 1, 2]),
            UBlock(512, 512, 5, [1, 2, 1, 2]),
            UBlock(512, 256, 3, [1, 2, 4, 8]),
            UBlock(256, 128, 2, [1, 2, 4, 8]),
            UBlock(128, 128, 2, [1, 2, 4, 8])])
        self.first_conv = Conv1d(128, 768, 3, padding=1)
        self.last_conv = Conv1d(128, 1, 3, padding=1)
        self.config_args = {}
        self.num_samples = -1
        self.compute_dtype = "float32"
        self._ctx = None
        self._ctx_key = None

    def library_config(self):
        return {"arch": {"type": "SDDM_spectrogram", "args": {"hop_samples": self.hop_samples}},
                "diffusion": {"type": "GaussianDiffusion", "args": {"schedule": "linear", "n_timestep": 1}},
                "network": {"type": "WaveGrad", "args": {}}, "num_samples": -1}

    def _context(self, device):
        sd = dict(self.state_dict())
        key = (device.index or 0, self.compute_dtype) + tuple((k, v.data_ptr(), v._version) for k, v in sd.items())
        if self._ctx is None or self._ctx_key != key:
            ctx = sddm_hip.Context(self.library_config(), device.index or 0, self.compute_dtype)
            ctx.load_state_dict(sd)
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    @torch.no_grad()
    def forward(self, spectrogram, audio, noise_scale):
        """spectrogram [B, 128, F], audio [B, 300 F] (or [B, 1, 300 F]), noise_scale [B] (any shape
        with B elements) -> squeeze(eps) (wavegrad.py:167-179)."""
        if not audio.is_cuda:
            raise RuntimeError("WaveGrad runs on the HIP device; move the tensors to cuda")
        B = spectrogram.shape[0]
        spec = spectrogram.contiguous().float()
        check_spectrogram(spec, self.freq_bins, "WaveGrad")
        x = audio.reshape(B, 1, -1).contiguous().float()
        nl = noise_scale.reshape(-1).contiguous().float()
        if nl.numel() != B:
            raise RuntimeError(f"noise_scale has {nl.numel()} elements for batch {B}")
        out = torch.empty_like(x)
        self._context(x.device).network_forward(spec, x, nl, out)
        return torch.squeeze(out)
