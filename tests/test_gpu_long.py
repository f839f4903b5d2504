"""GPU: the long sampling loops the benches run, pinned against the REFERENCE (tests/golden/long_loops.npz,
made by tests/golden/gen_golden.py --only long from /root/reference with the Philox stream injected).

  * UNetModified2 + SDDM.infer, condition_in, T=1000 (config_unet.json schedule linear 1e-6..1e-3 at the
    headline's step count; N=2112, B=2)                          model/model.py:50-124
  * DiffWave + SDDM_spectrogram.infer, T=200, time_step condition (config_diffwave.json; 63 frames, B=1)
                                                                  model/model.py:212-257
  * WaveGrad + SDDM_spectrogram.infer, T=50 (SURVEY §8d fast schedule; 54 frames, B=2: the reference
    WaveGrad cannot run one clip)

fp32 on the HIP path, north_star's bar: RMS <= 1e-3 against the reference output.  The reduced-precision
drift of config #5 (fp16, N=32832, fp32 GroupNorm statistics) over the full T=1000 loop is gated here
against the HIP fp32 path (itself pinned to the reference above): RMS <= 2e-3.
"""
import numpy as np
import pytest
import torch

import sddm_hip
from _helpers import diffwave_params, golden, rms, unet_config, unet_params, wavegrad_params

pytestmark = pytest.mark.gpu

LONG = "long_loops.npz"


def _unet_sample(ctx, cond_np, seed=7):
    dev = torch.device("cuda", 0)
    cond = torch.from_numpy(np.ascontiguousarray(cond_np)).to(dev)
    out = torch.full_like(cond, float("nan"))
    ctx.sample(cond, out, seed, 0)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _unet_ctx(N, dtype, sched):
    ctx = sddm_hip.Context(unet_config(N, sched), 0, dtype)
    for k, v in unet_params(N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    assert ctx.missing() == 0
    return ctx


def test_unet_condition_in_1000_steps_matches_reference(torch_cuda):
    z = golden(LONG)
    k = "long/unet/condition_in/linear_1000_1e-06_0.001/2112x2"
    out = _unet_sample(_unet_ctx(2112, "float32", ("linear", 1000, 1e-6, 1e-3)), z[f"{k}/cond"])
    ref = z[f"{k}/out"]
    err = rms(out, ref)
    print(f"UNet T=1000 fp32 vs reference: rms {err:.3e} (signal rms {rms(ref, 0):.3f}), "
          f"max |diff| {np.abs(out - ref).max():.3e}")
    assert np.isfinite(out).all()
    assert err <= 1e-3


def test_diffwave_200_steps_matches_reference(torch_cuda):
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    z = golden(LONG)
    k = "long/diffwave/time_step/linear_200_0.0001_0.02/63x1"
    net = NW.DiffWave(num_samples=-1, num_timesteps=200, freq_bins=513, residual_channels=64, residual_layers=30,
                      dilation_cycle_length=10)
    net.load_state_dict({n: torch.from_numpy(v) for n, v in diffwave_params().items()})
    d = D.GaussianDiffusion("linear", 200, 1e-4, 0.02, device="cuda")
    m = M.SDDM_spectrogram(d, net, hop_samples=256, noise_condition="time_step").cuda()
    out = m.infer(torch.from_numpy(z[f"{k}/spec"]).cuda(), seed=7).cpu().numpy()
    ref = z[f"{k}/out"]
    err = rms(out, ref)
    print(f"DiffWave T=200 fp32 vs reference: rms {err:.3e} (signal rms {rms(ref, 0):.3f})")
    assert out.shape == ref.shape and np.isfinite(out).all()
    assert err <= 1e-3


def test_wavegrad_50_steps_matches_reference(torch_cuda):
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    z = golden(LONG)
    k = "long/wavegrad/sqrt_alpha_bar/linear_50_0.0001_0.05/54x2"
    net = NW.WaveGrad()
    net.load_state_dict({n: torch.from_numpy(v) for n, v in wavegrad_params().items()})
    d = D.GaussianDiffusion("linear", 50, 1e-4, 0.05, device="cuda")
    m = M.SDDM_spectrogram(d, net, hop_samples=300).cuda()
    out = m.infer(torch.from_numpy(z[f"{k}/spec"]).cuda(), seed=7).cpu().numpy()
    ref = z[f"{k}/out"]
    err = rms(out, ref)
    print(f"WaveGrad T=50 fp32 vs reference: rms {err:.3e} (signal rms {rms(ref, 0):.3f})")
    assert out.shape == ref.shape and np.isfinite(out).all()
    assert err <= 1e-3


def test_config5_fp16_drift_1000_steps(torch_cuda):
    """Config #5's arithmetic (fp16 storage, fp32 accumulation and GroupNorm statistics) over the full
    T=1000 loop at its chunk length N=32832, 4 rows: drift against the HIP fp32 path."""
    from sddm_hip.synth import noisy_speech
    N, sched = 32832, ("linear", 1000, 1e-6, 1e-3)
    cond = noisy_speech(4, N, seed=77)
    out32 = _unet_sample(_unet_ctx(N, "float32", sched), cond)
    out16 = _unet_sample(_unet_ctx(N, "float16", sched), cond)
    err = rms(out16, out32)
    rows = [rms(out16[b], out32[b]) for b in range(4)]
    print(f"config #5 T=1000 fp16 vs fp32 (N={N}, 4 rows): rms {err:.3e}, worst row {max(rows):.3e}")
    assert np.isfinite(out16).all()
    assert err <= 2e-3
