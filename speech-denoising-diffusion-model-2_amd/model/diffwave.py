"""DiffWave facade (reference model/diffwave.py:22-155).

The module tree only *holds parameters*: names and shapes follow the reference so that
``state_dict()`` / ``load_state_dict`` exchange reference checkpoints unchanged (split=True
ResidualBlocks: output_residual + output_projection).  ``forward`` never computes in torch: the
upsampler, the 30 gated residual layers and the projections run as HIP kernels in libsddm_hip
(csrc/diffwave.hip).  ``DiffusionEmbedding.embedding_vector`` is built with torch's fp32 ops,
as in the reference (diffwave.py:25-28), and handed to the library.
"""
from math import sqrt  # noqa: F401  (reference import surface)

import torch
from torch import nn

import sddm_hip


def Conv1d(*args, **kwargs):
    layer = nn.Conv1d(*args, **kwargs)
    nn.init.kaiming_normal_(layer.weight)                          # diffwave.py:11-14
    return layer



def check_spectrogram(spec, bins, who):
    """The library reads [B, bins, F] with the configured bins; a different bin count would be read
    out of bounds.  The reference raises here too (its Conv1d(freq_bins, ...) rejects the shape)."""
    if spec.dim() != 3 or spec.shape[1] != bins:
        raise RuntimeError(f"{who} expects a spectrogram [B, {bins}, frames], got {tuple(spec.shape)}")

class DiffusionEmbedding(nn.Module):
    def __init__(self, dim=128):
        super().__init__()
        self.dim = dim
        step = torch.arange(self.dim // 2) / (self.dim // 2)
        self.embedding_vector = 10.0 ** (step * 4.0 / 63)         # diffwave.py:28 (not a buffer)
        self.projection1 = nn.Linear(128, 512)
        self.projection2 = nn.Linear(512, 512)


class SpectrogramUpsampler(nn.Module):
    def __init__(self, freq_bins):
        super().__init__()
        self.conv1 = nn.ConvTranspose2d(1, 1, [3, 32], stride=[1, 16], padding=[1, 8])
        self.conv2 = nn.ConvTranspose2d(1, 1, [3, 32], stride=[1, 16], padding=[1, 8])


class ResidualBlock(nn.Module):
    def __init__(self, freq_bins, residual_channels, dilation, fix_in=False, split=True):
        super().__init__()
        if not split:
            raise NotImplementedError("ResidualBlock(split=False): the reference DiffWave builds split=True")
        self.dilated_conv = Conv1d(residual_channels, 2 * residual_channels, 3, padding=dilation, dilation=dilation)
        self.diffusion_projection = nn.Linear(512, residual_channels)
        self.conditioner_projection = Conv1d(freq_bins, 2 * residual_channels, 1)
        self.split = split
        self.fix_in = fix_in
        self.output_projection = Conv1d(residual_channels, residual_channels, 1)
        self.output_residual = Conv1d(residual_channels, residual_channels, 1)


class DiffWave(nn.Module):
    def __init__(self, num_samples, num_timesteps, freq_bins, residual_channels=64, residual_layers=30,
                 dilation_cycle_length=10):
        super().__init__()
        self.num_samples = num_samples
        self.freq_bins = freq_bins
        self.config_args = {"residual_channels": residual_channels, "residual_layers": residual_layers,
                            "dilation_cycle_length": dilation_cycle_length, "freq_bins": freq_bins}
        self.input_projection = Conv1d(1, residual_channels, 1)
        self.diffusion_embedding = DiffusionEmbedding()
        self.spectrogram_upsampler = SpectrogramUpsampler(freq_bins)
        self.residual_layers = nn.ModuleList([
            ResidualBlock(freq_bins, residual_channels, 2 ** (i % dilation_cycle_length))
            for i in range(residual_layers)])
        self.skip_projection = Conv1d(residual_channels, residual_channels, 1)
        self.output_projection = Conv1d(residual_channels, 1, 1)
        nn.init.zeros_(self.output_projection.weight)                # diffwave.py:131
        self.compute_dtype = "float32"
        self._ctx = None
        self._ctx_key = None

    def library_params(self):
        """state_dict + the fp32 embedding vector (a plain attribute in the reference)."""
        sd = dict(self.state_dict())
        sd["diffusion_embedding.embedding_vector"] = self.diffusion_embedding.embedding_vector.float()
        return sd

    def library_config(self):
        return {"arch": {"type": "SDDM_spectrogram", "args": {"hop_samples": 256}},
                "diffusion": {"type": "GaussianDiffusion", "args": {"schedule": "linear", "n_timestep": 1}},
                "network": {"type": "DiffWave", "args": self.config_args}, "num_samples": self.num_samples}

    def _context(self, device):
        sd = self.library_params()
        key = (device.index or 0, self.compute_dtype) + tuple((k, v.data_ptr(), v._version) for k, v in sd.items())
        if self._ctx is None or self._ctx_key != key:
            ctx = sddm_hip.Context(self.library_config(), device.index or 0, self.compute_dtype)
            ctx.load_state_dict(sd)
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    @torch.no_grad()
    def forward(self, spectrogram, audio, diffusion_step):
        """spectrogram [B, bins, F], audio [B, 1, 256 F], diffusion_step [B, 1, 1] -> eps [B, 1, 256 F]
        (diffwave.py:133-155)."""
        if not audio.is_cuda:
            raise RuntimeError("DiffWave runs on the HIP device; move the tensors to cuda")
        spec = spectrogram.contiguous().float()
        check_spectrogram(spec, self.freq_bins, "DiffWave")
        x = audio.contiguous().float()
        nl = diffusion_step.reshape(-1).contiguous().float()
        out = torch.empty_like(x)
        self._context(x.device).network_forward(spec, x, nl, out)
        return out
