"""GPU: sampling with the reference's OWN noise (SURVEY §8(b) noise_mode 1, sddm_sample_noise).

tests/golden/torch_noise.npz was made by tests/golden/gen_golden.py --only torchnoise: the reference's
SDDM.infer / SDDM_spectrogram.infer run on CPU with torch.manual_seed(seed) and NO noise injection, so
every draw is the reference's torch.randn_like / torch.randn (model.py:57-68,216;
diffusion.py:172,187,207,220,285,306).  Here model.model.reference_noise() re-draws them from the same
seed on the CPU generator in the reference's order and the HIP loop consumes them through
sddm_sample_noise: fp32 RMS <= 1e-5 against the reference output, for all five p_transition modes
(UNetModified2, T=6) and DiffWave (T=6, time_step condition).
"""
import numpy as np
import pytest
import torch

from _helpers import UNET_NET, diffwave_params, golden, parse_sched_key, rms, unet_params

pytestmark = pytest.mark.gpu

TN = "torch_noise.npz"
MODES = ("condition_in", "original", "sr3", "supportive", "conditional")


@pytest.mark.parametrize("mode", MODES)
def test_unet_sampling_with_reference_torch_noise(torch_cuda, mode):
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    z = golden(TN)
    key = [k.rsplit("/", 1)[0] for k in z.files if k.startswith(f"torchnoise/unet/{mode}/") and k.endswith("/out")][0]
    sched = parse_sched_key(key.split("/")[3])
    N = int(key.split("/")[4].split("x")[0])
    dev = torch.device("cuda", 0)
    net = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in unet_params(N).items()})
    m = M.SDDM(D.GaussianDiffusion(*sched, device=dev), net, p_transition=mode).to(dev)
    cond = torch.from_numpy(z[key + "/cond"])
    torch.manual_seed(int(z[key + "/seed"]))
    noise = M.reference_noise(m, cond, device="cpu")
    out = m.infer(cond.to(dev), noise=noise).cpu().numpy()
    ref = z[key + "/out"]
    err = rms(out, ref)
    print(f"{mode} T={sched[1]} with the reference's torch noise: rms {err:.3e} (signal rms {rms(ref, 0):.3f})")
    assert np.isfinite(out).all() and err <= 1e-5


def test_diffwave_sampling_with_reference_torch_noise(torch_cuda):
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    z = golden(TN)
    key = [k.rsplit("/", 1)[0] for k in z.files if k.startswith("torchnoise/diffwave/") and k.endswith("/out")][0]
    sched = parse_sched_key(key.split("/")[3])
    net = NW.DiffWave(num_samples=-1, num_timesteps=sched[1], freq_bins=513, residual_channels=64, residual_layers=30,
                      dilation_cycle_length=10)
    net.load_state_dict({n: torch.from_numpy(v) for n, v in diffwave_params().items()})
    dev = torch.device("cuda", 0)
    m = M.SDDM_spectrogram(D.GaussianDiffusion(*sched, device=dev), net, hop_samples=256,
                           noise_condition="time_step").to(dev)
    spec = torch.from_numpy(z[key + "/spec"])
    torch.manual_seed(int(z[key + "/seed"]))
    noise = M.reference_noise(m, spec, device="cpu")
    out = m.infer(spec.to(dev), noise=noise).cpu().numpy()
    ref = z[key + "/out"]
    err = rms(out, ref)
    print(f"DiffWave T={sched[1]} with the reference's torch noise: rms {err:.3e} (signal rms {rms(ref, 0):.3f})")
    assert out.shape == ref.shape and np.isfinite(out).all() and err <= 1e-5


def test_reference_noise_layout_and_errors(torch_cuda):
    """reference_noise draws x_T (none for 'supportive') then t = T .. 2; a wrongly shaped buffer raises."""
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    N, sched = 2112, ("linear", 4, 1e-4, 0.05)
    net = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    cond = torch.zeros(2, 1, N)
    for mode in ("original", "supportive"):
        m = M.SDDM(D.GaussianDiffusion(*sched, device="cpu"), net, p_transition=mode)
        torch.manual_seed(3)
        nz = M.reference_noise(m, cond, device="cpu")
        assert nz.shape == (5, 2, 1, N) and float(nz[1].abs().max()) == 0.0
        torch.manual_seed(3)
        first = torch.randn(2, 1, N)
        assert torch.equal(nz[0 if mode == "original" else 4], first)
    m = M.SDDM(D.GaussianDiffusion(*sched, device="cuda"), net).to("cuda")
    net.load_state_dict({k: torch.from_numpy(v) for k, v in unet_params(N).items()})
    with pytest.raises(ValueError):
        m.infer(cond.cuda(), noise=torch.zeros(3, 2, 1, N))


def test_sample_noise_checks_default_timesteps(torch_cuda):
    """A library config without n_timestep runs the library's default T = 1000 (sddm_configure), so
    the Context checks a caller noise buffer against 1001 draws: a shorter one raises instead of
    letting the library read past its end."""
    import sddm_hip
    from _helpers import unet_config
    N = 2112
    cfg = unet_config(N, ("linear", 4, 1e-4, 0.05))
    del cfg["diffusion"]["args"]["n_timestep"]
    ctx = sddm_hip.Context(cfg, 0, "float32")
    assert ctx.timesteps == 1000
    cond = torch.zeros(1, 1, N, device="cuda")
    with pytest.raises(ValueError):
        ctx.sample_noise(cond, torch.empty_like(cond), torch.zeros(5, 1, 1, N, device="cuda"))


def test_unet_caller_noise_across_lanes(torch_cuda):
    """Caller noise with B larger than the lane (lane_rows = 2, B = 4: two lanes, each reading its rows
    of every draw at noise + row0 * N with stride B * N, final_kernel's vector noise loads included):
    the HIP loop equals the oracle fed the same draws (fp32, T=3, distinct rows)."""
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    from oracle import sampler, unet
    from oracle.schedule import BUFFER_NAMES
    from sddm_hip.synth import noisy_speech
    N, B, sched = 2112, 4, ("linear", 3, 1e-4, 0.05)
    dev = torch.device("cuda", 0)
    P = unet_params(N)
    net = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    d = D.GaussianDiffusion(*sched, device=dev)
    m = M.SDDM(d, net, p_transition="original").to(dev)
    m.lane_rows = 2
    cond = noisy_speech(B, N, seed=11)
    noise = np.random.default_rng(5).standard_normal((sched[1] + 1, B, 1, N)).astype(np.float32)
    out = m.infer(torch.from_numpy(cond).to(dev), noise=torch.from_numpy(noise)).cpu().numpy()
    tab = {k: getattr(d, k).cpu().numpy() for k in BUFFER_NAMES}
    arch = unet.architecture(N, inner_channel=32, channel_mults=(1, 2, 3, 4, 5), res_blocks=1)
    ref = sampler.infer(lambda c, x, nl: unet.forward(P, arch, c, x, nl), tab, cond, "original", noise=noise)
    errs = [rms(out[b], ref[b]) for b in range(B)]
    print(f"caller noise, 2-row lanes x 2: row rms {' '.join(f'{e:.2e}' for e in errs)}")
    assert np.isfinite(out).all() and max(errs) <= 1e-5


def test_wavegrad_caller_noise_matches_oracle(torch_cuda):
    """SDDM_spectrogram.infer + WaveGrad with caller draws (sddm_sample_noise on the WaveGrad loop)
    equals the oracle's infer_spectrogram fed the same draws (fp32, T=3, B=2, 6 frames)."""
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    from oracle import sampler
    from oracle import wavegrad as wg
    from oracle.schedule import BUFFER_NAMES
    from _helpers import wavegrad_params
    sched = ("linear", 3, 1e-4, 0.05)
    dev = torch.device("cuda", 0)
    P = wavegrad_params()
    net = NW.WaveGrad()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    d = D.GaussianDiffusion(*sched, device=dev)
    m = M.SDDM_spectrogram(d, net.to(dev), hop_samples=300).to(dev)
    rng = np.random.default_rng(9)
    spec = rng.uniform(0, 1, (2, 128, 6)).astype(np.float32)
    noise = rng.standard_normal((sched[1] + 1, 2, 1, 300 * 6)).astype(np.float32)
    out = m.infer(torch.from_numpy(spec).to(dev), noise=torch.from_numpy(noise)).cpu().numpy()
    tab = {k: getattr(d, k).cpu().numpy() for k in BUFFER_NAMES}
    ref = sampler.infer_spectrogram(lambda s, x, nl: wg.forward(P, s, x.reshape(x.shape[0], -1), nl).reshape(x.shape),
                                    tab, spec, 300, noise=noise)
    err = rms(out, ref)
    print(f"WaveGrad caller noise: rms {err:.3e} (signal rms {rms(ref, 0):.3f})")
    assert out.shape == ref.shape and np.isfinite(out).all() and err <= 1e-4 * max(1.0, rms(ref, 0))
