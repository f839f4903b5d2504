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
