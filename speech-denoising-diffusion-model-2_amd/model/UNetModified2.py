"""UNetModified2 facade (reference model/UNetModified2.py:146-269).

The module tree only *holds parameters*, laid out so that ``state_dict()`` has exactly the
reference's keys and shapes (232 entries with the diffusion buffers at config_unet.json), and
``load_state_dict`` accepts a reference checkpoint unchanged.  ``forward`` never computes in
torch: it hands the weights to libsddm_hip and runs the whole denoiser as HIP kernels
(framing, MFMA convolutions with fused GroupNorm/SiLU, embedding MLP, overlap-add).
"""
import torch
from torch import nn

import sddm_hip


class SignalToFrames(nn.Module):
    """Framing geometry of UNetModified2.py:5-28 (idx[f, w] = stride * f + w)."""

    def __init__(self, n_samples, F=512, stride=256):
        super().__init__()
        assert (n_samples - F) % stride == 0                                    # UNetModified2.py:13
        self.n_samples, self.F, self.stride = n_samples, F, stride
        self.n_frames = (n_samples - F) // stride + 1
        self.idx_mat = torch.arange(self.n_frames)[:, None] * stride + torch.arange(F)[None, :]


class Swish(nn.Module):
    pass


class PositionalEncoding(nn.Module):
    """UNetModified2.py:49-55: fp32 1e4 * 10 ** (-k * 4 / half)."""

    def __init__(self, dim=128):
        super().__init__()
        self.dim = dim
        half = dim // 2
        self.embedding_vector = 1e4 * 10.0 ** (-torch.arange(half) * 4.0 / half)


class FeatureWiseAffine(nn.Module):
    def __init__(self, in_channels, out_channels, use_affine_level=False):
        super().__init__()
        if use_affine_level:
            raise NotImplementedError("use_affine_level=True is never used by UNetModified2 (UNetModified2.py:128)")
        self.use_affine_level = use_affine_level
        self.noise_func = nn.Sequential(nn.Linear(in_channels, out_channels))


class Block(nn.Module):
    """GroupNorm -> Swish -> (Dropout) -> Conv3x3 (UNetModified2.py:113-124)."""

    def __init__(self, dim, dim_out, groups=32, dropout=0):
        super().__init__()
        self.block = nn.Sequential(nn.GroupNorm(groups, dim), Swish(),
                                   nn.Dropout(dropout) if dropout != 0 else nn.Identity(),
                                   nn.Conv2d(dim, dim_out, 3, padding=1))


class ResnetBlock(nn.Module):
    def __init__(self, dim, dim_out, noise_level_emb_dim, dropout=0, norm_groups=32, use_affine_level=False):
        super().__init__()
        self.noise_func = FeatureWiseAffine(noise_level_emb_dim, dim_out, use_affine_level)
        self.block1 = Block(dim, dim_out, groups=norm_groups)
        self.block2 = Block(dim_out, dim_out, groups=norm_groups, dropout=dropout)
        self.res_conv = nn.Conv2d(dim, dim_out, 1) if dim != dim_out else nn.Identity()


class Upsample(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.up = nn.Upsample(scale_factor=2, mode="nearest")
        self.conv = nn.Conv2d(dim, dim, 3, padding=1)


class Downsample(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.conv = nn.Conv2d(dim, dim, 3, 2, 1)


class UNetModified2(nn.Module):
    def __init__(self, num_samples, in_channel=2, out_channel=1, inner_channel=32, norm_groups=32,
                 channel_mults=(1, 2, 3, 4, 5), res_blocks=3, dropout=0, segment_len=128, segment_stride=64):
        super().__init__()
        self.num_samples = num_samples
        self.config_args = {"in_channel": in_channel, "out_channel": out_channel, "inner_channel": inner_channel,
                            "norm_groups": norm_groups, "channel_mults": list(channel_mults),
                            "res_blocks": res_blocks, "dropout": dropout, "segment_len": segment_len,
                            "segment_stride": segment_stride}
        self.segment = SignalToFrames(num_samples, segment_len, segment_stride)
        E = inner_channel
        self.noise_level_mlp = nn.Sequential(PositionalEncoding(E), nn.Linear(E, E * 4), Swish(),
                                             nn.Linear(E * 4, E), Swish())
        rb = dict(noise_level_emb_dim=E, norm_groups=norm_groups, dropout=dropout)
        downs = [nn.Conv2d(in_channel, E, kernel_size=3, padding=1)]
        skip = [E]
        cin = E
        for mult in channel_mults:                                   # encoder (UNetModified2.py:186-198)
            cout = E * mult
            for _ in range(res_blocks):
                downs.append(ResnetBlock(cin, cout, **rb))
                skip.append(cout)
                cin = cout
            downs.append(Downsample(cout))
            skip.append(cout)
        self.downs = nn.ModuleList(downs)
        self.mid = nn.ModuleList([ResnetBlock(cin, cin, **rb)])
        ups = []
        for ind in reversed(range(len(channel_mults))):               # decoder (UNetModified2.py:208-232)
            cin = E * channel_mults[ind]
            ups.append(ResnetBlock(cin + skip.pop(), cin, **rb))
            ups.append(Upsample(cin))
            cout = E if ind == 0 else E * channel_mults[ind - 1]
            for _ in range(res_blocks):
                ups.append(ResnetBlock(cin + skip.pop(), cout, **rb))
                cin = cout
        self.ups = nn.ModuleList(ups)
        self.final_conv = Block(cout, out_channel, groups=norm_groups)
        self.compute_dtype = "float32"
        self._ctx = None
        self._ctx_key = None

    def library_config(self):
        return {"arch": {"type": "SDDM", "args": {}},
                "diffusion": {"type": "GaussianDiffusion", "args": {"schedule": "linear", "n_timestep": 1}},
                "network": {"type": "UNetModified2", "args": self.config_args},
                "num_samples": self.num_samples}

    def _context(self, device):
        sd = self.state_dict()
        key = (device.index or 0, self.compute_dtype) + tuple((k, v.data_ptr(), v._version) for k, v in sd.items())
        if self._ctx is None or self._ctx_key != key:
            ctx = sddm_hip.Context(self.library_config(), device.index or 0, self.compute_dtype)
            ctx.load_state_dict(sd)
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    @torch.no_grad()
    def forward(self, x, y_t, diffusion_step):
        """x: condition [B,1,T], y_t: [B,1,T], diffusion_step: noise level [B,1,1] -> eps [B,1,T]."""
        if not x.is_cuda:
            raise RuntimeError("UNetModified2 runs on the HIP device; move inputs to cuda")
        x = x.contiguous().float()
        y_t = y_t.contiguous().float()
        nl = diffusion_step.reshape(-1).contiguous().float()
        if nl.numel() == 1 and x.shape[0] > 1:
            nl = nl.expand(x.shape[0]).contiguous()
        out = torch.empty_like(y_t)
        self._context(x.device).network_forward(x, y_t, nl, out)
        return out
