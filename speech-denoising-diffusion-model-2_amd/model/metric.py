"""Metrics (reference model/metric.py:5-34): scale-invariant SNR."""
import torch


def sisnr(s_hat, s):
    """SI-SNR in dB averaged over the batch; s_hat, s: [B, 1, T] or [B, T]."""
    if s_hat.ndim == 2:
        s_hat = torch.unsqueeze(s_hat, 1)
    if s.ndim == 2:
        s = torch.unsqueeze(s, 1)
    s_hat = s_hat - torch.mean(s_hat, dim=-1, keepdim=True)
    s = s - torch.mean(s, dim=-1, keepdim=True)
    s_target = torch.sum(s_hat * s, dim=-1, keepdim=True) * s / torch.sum(s ** 2, dim=-1, keepdim=True)
    e_noise = s_hat - s_target
    v = 10 * torch.log10(torch.sum(s_target ** 2, dim=-1, keepdim=True) / torch.sum(e_noise ** 2, dim=-1, keepdim=True))
    return torch.squeeze(torch.mean(v))
