"""GPU: the drop-in facade (model.model.SDDM, model.diffusion.GaussianDiffusion,
model.network.UNetModified2) reproduces the reference goldens through libsddm_hip."""
import numpy as np
import pytest
import torch

from _helpers import UNET_NET, golden, parse_sched_key, rms, unet_params

pytestmark = pytest.mark.gpu


def _model(N, sched, mode="condition_in", dtype="float32"):
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    dev = torch.device("cuda", 0)
    d = D.GaussianDiffusion(*sched, device=dev)
    n = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    n.load_state_dict({k: torch.from_numpy(v) for k, v in unet_params(N).items()})
    return M.SDDM(d, n, p_transition=mode, compute_dtype=dtype).to(dev)


def test_sddm_infer_facade_matches_reference(torch_cuda):
    inf = golden("unet_infer.npz")
    key = "inf/condition_in/linear_4_1e-06_0.001/2112x2"
    m = _model(2112, parse_sched_key("linear_4_1e-06_0.001"))
    out = m.infer(torch.from_numpy(inf[key + "/cond"]).cuda(), seed=7).cpu().numpy()
    assert rms(out, inf[key + "/out"]) <= 1e-3


def test_continuous_sampling_records_every_inter_step(torch_cuda):
    inf = golden("unet_infer.npz")
    key = "inf/condition_in/linear_4_1e-06_0.001/2112x2"
    m = _model(2112, parse_sched_key("linear_4_1e-06_0.001"))
    cond = torch.from_numpy(inf[key + "/cond"][:1]).cuda()
    samples = m.infer(cond, continuous=True, seed=7)
    assert len(samples) == 1 + 4 and samples[0] is cond          # [condition] + x_3, x_2, x_1, x_0
    steps = inf[key + "/steps"][:, :1]
    got = np.stack([s.cpu().numpy() for s in samples[1:]])
    assert rms(got, steps) <= 1e-3
    with pytest.raises(AssertionError):
        m.infer(torch.from_numpy(inf[key + "/cond"]).cuda(), continuous=True)   # model.py:80


def test_diffusion_facade_transitions(torch_cuda):
    import model.diffusion as D
    tr = golden("transitions.npz")
    d = D.GaussianDiffusion("linear", 100, 1e-6, 1e-3, device="cuda")
    base = "tr/linear_100_1e-06_0.001"
    for mode, fn in (("original", d.p_transition), ("sr3", d.p_transition_sr3)):
        k = f"{base}/{mode}/50"
        x, e = (torch.from_numpy(tr[f"{k}/{n}"]).cuda() for n in ("x_t", "eps"))
        assert np.abs(fn(x, 50, e, seed=7).cpu().numpy() - tr[f"{k}/out"]).max() <= 2e-6
    for mode, fn in (("supportive", d.p_transition_supportive), ("conditional", d.p_transition_conditional)):
        k = f"{base}/{mode}/50"
        x, e, c = (torch.from_numpy(tr[f"{k}/{n}"]).cuda() for n in ("x_t", "eps", "cond"))
        out = fn(x, 50, e, c, seed=7).cpu().numpy()
        assert np.allclose(out, tr[f"{k}/out"], atol=2e-6, rtol=0, equal_nan=True)
    c = torch.from_numpy(tr[f"{base}/get_x_T/cond"]).cuda()
    assert np.abs(d.get_x_T(c, seed=7).cpu().numpy() - tr[f"{base}/get_x_T/out"]).max() <= 2e-6


def test_unet_facade_forward(torch_cuda):
    import model.network as NW
    fw = golden("unet_forward.npz")
    N = 2112
    n = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    n.load_state_dict({k: torch.from_numpy(v) for k, v in unet_params(N).items()})
    n = n.cuda()
    eps = n(torch.from_numpy(fw[f"fw/{N}/cond"]).cuda(), torch.from_numpy(fw[f"fw/{N}/x_t"]).cuda(),
            torch.from_numpy(fw[f"fw/{N}/noise_level"]).reshape(-1, 1, 1).cuda())
    assert rms(eps.cpu().numpy(), fw[f"fw/{N}/eps"]) <= 1e-4
    # weights changed in place -> the library copy is refreshed
    with torch.no_grad():
        n.final_conv.block[3].bias.add_(1.0)
    eps2 = n(torch.from_numpy(fw[f"fw/{N}/cond"]).cuda(), torch.from_numpy(fw[f"fw/{N}/x_t"]).cuda(),
             torch.from_numpy(fw[f"fw/{N}/noise_level"]).reshape(-1, 1, 1).cuda())
    assert float((eps2 - eps).abs().mean()) > 0.5


def test_geometry_errors_raise_like_reference(torch_cuda):
    import model.network as NW
    # n_frames = 249 is not a multiple of 32: the reference fails at torch.cat (shape error)
    n = NW.UNetModified2(num_samples=16000, **UNET_NET["args"]).cuda()
    x = torch.zeros(1, 1, 16000, device="cuda")
    with pytest.raises(AssertionError):
        n(x, x, torch.ones(1, 1, 1, device="cuda"))
    m = _model(2112, ("linear", 4, 1e-6, 1e-3))
    with pytest.raises(AssertionError):
        m.infer(torch.zeros(1, 1, 2176, device="cuda"))        # condition length != num_samples


def test_bf16_sampling_close_to_fp32(torch_cuda):
    inf = golden("unet_infer.npz")
    key = "inf/condition_in/linear_50_1e-06_0.001/16448x1"
    m = _model(16448, parse_sched_key("linear_50_1e-06_0.001"), dtype="bfloat16")
    out = m.infer(torch.from_numpy(inf[key + "/cond"]).cuda(), seed=7).cpu().numpy()
    err = rms(out, inf[key + "/out"])
    print("bf16 50-step rms vs fp32 reference", err)
    assert err <= 1e-2     # bf16 network storage: stated tolerance


@pytest.mark.parametrize("q_transition,noise_condition", [("original", "sqrt_alpha_bar"), ("original", "time_step"),
                                                          ("conditional", "sqrt_alpha_bar")])
def test_sddm_forward_training_step(torch_cuda, q_transition, noise_condition):
    """SDDM.forward (model.py:29-48): q-sample on HIP, then the network on HIP, against the oracle's
    q_stochastic* (diffusion.py:225-279, pinned by q_sample.npz) composed with oracle/unet.forward
    (pinned by unet_forward.npz), with the reference's draws (randint / rand) made explicit."""
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    from oracle import sampler as osamp, unet as ounet
    from oracle.schedule import BUFFER_NAMES
    from _helpers import unet_arch
    from sddm_hip.synth import noisy_speech
    N, B, T = 2112, 3, 100
    dev = torch.device("cuda", 0)
    d = D.GaussianDiffusion("linear", T, 1e-6, 1e-3, device=dev)
    n = NW.UNetModified2(num_samples=N, **UNET_NET["args"])
    P = unet_params(N)
    n.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    m = M.SDDM(d, n, noise_condition=noise_condition, q_transition=q_transition).to(dev)
    target = noisy_speech(B, N, seed=11)
    cond = noisy_speech(B, N, seed=12)
    rng = np.random.default_rng(3)
    noise = rng.standard_normal(target.shape).astype(np.float32)
    t = np.array([1, 37, T], dtype=np.int64)
    r = rng.random(B).astype(np.float32)
    tab = {k: getattr(d, k).cpu().numpy() for k in BUFFER_NAMES}
    tg = lambda a: torch.from_numpy(a).to(dev)
    with pytest.raises(NotImplementedError):         # no HIP backward: grad mode refused
        m(tg(target), tg(cond), noise=tg(noise), t=tg(t), random_step=tg(r))
    if q_transition == "original":
        with torch.no_grad():
            pred, nz = m(tg(target), tg(cond), noise=tg(noise), t=tg(t), random_step=tg(r))
        x_t, s, level = osamp.q_stochastic(tab, target, noise, t, r)
        nl = s if noise_condition == "sqrt_alpha_bar" else level
        ref_noise = noise
    else:
        with torch.no_grad():
            pred, nz = m(tg(target), tg(cond), noise=tg(noise), t=tg(t.reshape(B, 1, 1)))
        x_t, ref_noise, nl = osamp.q_stochastic_conditional(tab, target, cond, noise, t)
    ref = ounet.forward(P, unet_arch(N), cond, x_t, np.asarray(nl, np.float32).reshape(-1))
    assert pred.shape == (B, 1, N) and nz.shape == (B, 1, N)
    assert np.abs(nz.cpu().numpy() - ref_noise).max() <= 1e-5
    assert rms(pred.cpu().numpy(), ref) <= 1e-4 * max(1.0, float(np.sqrt(np.mean(ref.astype(np.float64) ** 2))))
    with torch.no_grad(), pytest.raises(RuntimeError):
        m(tg(target).cpu(), tg(cond).cpu())
