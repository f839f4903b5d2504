"""Oracle pinning (CPU): the numpy restatement against the reference-generated golden vectors
and published known-answer vectors.  Parity of the HIP path is then checked against the same
fixtures / the oracle in the gpu tests."""
import numpy as np
import pytest

from oracle import philox, sampler, schedule, unet
from _helpers import golden, parse_sched_key, rms, tables_from_golden, unet_arch, unet_params

# Random123 kat_vectors for philox4x32_10
KAT = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
       ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
       ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
        (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_known_answers(ctr, key, expect):
    out = philox.philox4x32_10(*[np.array([c], dtype=np.uint64) for c in ctr], *key)
    assert tuple(int(o[0]) for o in out) == expect


def test_normal_stream_statistics_and_sharding():
    z = philox.normal(7, 3, (8, 1, 4096))
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1.0) < 0.02
    # rows sampled with a row offset equal the same rows of the full tensor
    assert np.array_equal(philox.normal(7, 3, (3, 1, 4096), row_offset=5), z[5:8])
    assert not np.array_equal(philox.normal(7, 4, (1, 1, 64)), philox.normal(7, 3, (1, 1, 64)))


def _sched_keys():
    S = golden("schedules.npz")
    return sorted({k.split("/")[1] for k in S.files})


@pytest.mark.parametrize("key", _sched_keys())
def test_schedule_tables(key):
    """betas / alphas / alpha_bar bit-exact (linspace + cumprod rules) for linear/quad; the rest
    within the few-ulp inaccuracy of torch's CPU sqrt/cos (diffusion.py:50-161)."""
    ref = tables_from_golden(key)
    mine = schedule.make_tables(*parse_sched_key(key))
    name = parse_sched_key(key)[0]
    for k in schedule.BUFFER_NAMES:
        r, m = ref[k], mine[k]
        assert np.array_equal(np.isnan(r), np.isnan(m)), k
        ok = ~np.isnan(r)
        if name != "cosine" and k in ("betas", "alphas", "alpha_bar"):
            assert np.array_equal(r.view(np.uint32), m.view(np.uint32)), k
        elif k in ("c_xt", "c_yt", "c_epst", "m", "sqrt_delta", "sqrt_delta_estimated", "supportive_sigma_hat"):
            # differences of nearly equal terms (conditional coefficients near delta ~ 0, Q8;
            # sigma - gamma / sqrt(alpha)): ulp-level input differences are amplified
            rel = np.abs(r[ok] - m[ok]) / np.maximum(np.abs(r[ok]), 1e-3)
            assert rel.max() <= 2e-2, (k, rel.max())
        elif name == "cosine":   # torch's fp32 cos differs by ulps; 1 - ab[t]/ab[t-1] cancels
            assert np.allclose(m[ok], r[ok], rtol=5e-3, atol=2e-6), k
        else:
            rel = np.abs(r[ok] - m[ok]) / np.maximum(np.abs(r[ok]), 1e-30)
            assert rel.max() <= 3e-7, (k, rel.max())


def test_embedding_vector_bit_exact():
    ref = golden("embedding.npz")["unet_embedding_vector"]
    assert np.array_equal(unet.embedding_vector(32).view(np.uint32), ref.view(np.uint32))


def test_transitions_bit_exact():
    tr = golden("transitions.npz")
    for key in sorted({k.rsplit("/", 1)[0] for k in tr.files}):
        parts = key.split("/")
        tab = tables_from_golden(parts[1])
        mode = parts[2]
        if mode.startswith("get_x_T"):
            z = philox.normal(7, 0, tr[key + "/cond"].shape)
            fn = sampler.get_x_T if mode == "get_x_T" else sampler.get_x_T_conditional
            out = fn(tab, tr[key + "/cond"], z)
        else:
            t = int(parts[3])
            z = philox.normal(7, t, tr[key + "/x_t"].shape) if t > 1 else None
            out = sampler.transition(mode, tab, tr[key + "/x_t"], t, tr[key + "/eps"], tr[key + "/cond"], z)
        ref = tr[key + "/out"]
        assert np.array_equal(np.isnan(out), np.isnan(ref)), key
        assert np.allclose(out, ref, rtol=0, atol=1e-6, equal_nan=True), key


@pytest.mark.parametrize("N", [2112, 16448])
def test_unet_forward_matches_reference(N):
    fw = golden("unet_forward.npz")
    P = unet_params(N)
    eps = unet.forward(P, unet_arch(N), fw[f"fw/{N}/cond"], fw[f"fw/{N}/x_t"], fw[f"fw/{N}/noise_level"])
    assert rms(eps, fw[f"fw/{N}/eps"]) <= 1e-5


def test_sampling_loops_match_reference():
    inf = golden("unet_infer.npz")
    for key in sorted({k.rsplit("/", 1)[0] for k in inf.files}):
        _, mode, sk, shp = key.split("/")
        N, B = map(int, shp.split("x"))
        if N > 2112:
            continue  # 50 full-size steps: covered on the GPU (test_gpu_unet.py)
        P = unet_params(N)
        arch = unet_arch(N)
        rec = []
        out = sampler.infer(lambda c, x, nl: unet.forward(P, arch, c, x, nl), tables_from_golden(sk),
                            inf[key + "/cond"], mode=mode, seed=7, record=rec)
        assert rms(out, inf[key + "/out"]) <= 1e-5, key
        steps = inf[key + "/steps"]
        assert rms(np.stack(rec[1:]), steps) <= 1e-5, key


def test_frame_index_and_overlap_add():
    """SignalToFrames / overlapAdd (UNetModified2.py:13-41): OLA of framed ones counts coverage."""
    idx = unet.frame_index(2112, 128, 64)
    assert idx.shape == (32, 128) and idx[1, 0] == 64 and idx[-1, -1] == 2111
    cover = unet.overlap_add(np.ones((1, 1, 32, 128), np.float32), 2112, 64)[0, 0]
    assert cover[:64].tolist() == [1.0] * 64 and cover[-64:].tolist() == [1.0] * 64
    assert (cover[64:-64] == 2.0).all()


# ---------------- DiffWave (reference model/diffwave.py) ----------------
def test_diffwave_oracle_matches_reference_goldens():
    from oracle import diffwave as dw
    from _helpers import diffwave_params
    z = golden("diffwave.npz")
    e = golden("embedding.npz")["diffwave_embedding_vector"]
    ulp = np.abs(dw.embedding_vector() - e) / np.spacing(e)
    assert ulp.max() <= 1.0                     # torch's fp32 pow (SLEEF) vs correctly rounded
    P = diffwave_params()
    k = "dw/fw/6x2"
    assert np.abs(dw.upsample(P, z[f"{k}/spec"])[:, :64] - z[f"{k}/upsampled"]).max() <= 1e-6
    eps = dw.forward(P, z[f"{k}/spec"], z[f"{k}/audio"], z[f"{k}/step"])
    assert np.sqrt(np.mean((eps - z[f"{k}/eps"]) ** 2)) <= 1e-6


def test_diffwave_oracle_sampling_matches_reference():
    from oracle import diffwave as dw, sampler
    from _helpers import diffwave_params, tables_from_golden
    z = golden("diffwave.npz")
    P = diffwave_params()
    sk = "linear_3_0.0001_0.05"
    k = f"dw/inf/time_step/{sk}/6x2"
    tab = tables_from_golden(sk)
    out = sampler.infer_spectrogram(lambda s, x, nl: dw.forward(P, s, x, nl), tab, z[f"{k}/spec"], 256,
                                    noise_condition="time_step", seed=7)
    assert np.sqrt(np.mean((out - z[f"{k}/out"]) ** 2)) <= 1e-5


# ---------------- WaveGrad (reference model/wavegrad.py) ----------------
def test_wavegrad_oracle_matches_reference_goldens():
    from oracle import wavegrad as wg
    from _helpers import wavegrad_params
    z = golden("wavegrad.npz")
    k = "wg/fw/6x2"
    eps = wg.forward(wavegrad_params(), z[f"{k}/spec"], z[f"{k}/audio"], z[f"{k}/noise_level"])
    assert eps.shape == z[f"{k}/eps"].shape
    assert rms(eps, z[f"{k}/eps"]) <= 1e-6


def test_wavegrad_param_shapes_match_reference_state_dict():
    import json
    import os
    from oracle import wavegrad as wg
    here = os.path.join(os.path.dirname(__file__), "golden", "state_dict_keys.json")
    keys = json.load(open(here))["wavegrad"]
    assert {k: tuple(s) for k, s in keys} == wg.param_shapes()


def test_wavegrad_oracle_sampling_matches_reference():
    """SDDM_spectrogram loop with the SURVEY Q4 adapter (eps [B,N] -> [B,1,N])."""
    from oracle import wavegrad as wg
    from _helpers import wavegrad_params
    z = golden("wavegrad.npz")
    P = wavegrad_params()
    sk = "linear_3_0.0001_0.05"
    k = f"wg/inf/sqrt_alpha_bar/{sk}/6x2"
    tab = tables_from_golden(sk)
    out = sampler.infer_spectrogram(lambda s, x, nl: wg.forward(P, s, x[:, 0], nl)[:, None], tab, z[f"{k}/spec"],
                                    wg.HOP, noise_condition="sqrt_alpha_bar", seed=7)
    assert rms(out, z[f"{k}/out"]) <= 1e-5


# ---------------- forward process q_stochastic (diffusion.py:225-279) ----------------
def _q_draws(T, B, seed, integer=False, cond=False):
    import torch
    torch.manual_seed(seed)
    if cond:
        return torch.randint(1, T + 1, (B, 1, 1)).reshape(-1).numpy(), None
    t = torch.randint(1, T + 1, [B]).numpy()
    return t, (None if integer else torch.rand(B).numpy())


@pytest.mark.parametrize("sk", ["linear_50_1e-06_0.001", "linear_200_0.0001_0.02"])
def test_q_stochastic_oracle_matches_reference(sk):
    z = golden("q_sample.npz")
    tab = tables_from_golden(sk)
    T = parse_sched_key(sk)[1]
    k = f"q/{sk}"
    x0, y, noise = z[k + "/x0"], z[k + "/y"], z[k + "/noise"]
    for name, integer in (("float", False), ("int", True)):
        t, r = _q_draws(T, x0.shape[0], 5, integer)
        x_t, s, lvl = sampler.q_stochastic(tab, x0, noise, t, r)
        assert np.abs(x_t - z[f"{k}/{name}/x_t"]).max() <= 1e-6
        assert np.array_equal(s, z[f"{k}/{name}/s"].reshape(-1))
        assert np.array_equal(lvl, z[f"{k}/{name}/level"].reshape(-1))
    t, _ = _q_draws(T, x0.shape[0], 6, cond=True)
    x_t, comb, s = sampler.q_stochastic_conditional(tab, x0, y, noise, t)
    ok = np.isfinite(z[f"{k}/cond/x_t"])
    assert np.abs(x_t - z[f"{k}/cond/x_t"])[ok].max() <= 1e-6
    assert np.abs(comb - z[f"{k}/cond/combined"])[ok].max() <= 1e-5


# ---------------- spectrogram featurizer (prepare_spectrogram.py:20-55) ----------------
def test_featurizer_oracle_matches_stft_fixture():
    from oracle import features as fe
    z = golden("stft.npz")
    assert np.abs(fe.hamming(1024) - z["stft/window"]).max() <= 1e-6
    assert np.abs(fe.hann(1024) - z["stft/window_mel"]).max() <= 1e-6
    for name, fb in (("spec", None), ("mel", z["stft/fb"])):
        out = fe.log_spectrogram(z["stft/audio"], fb=fb)
        assert out.shape == z[f"stft/{name}"].shape
        assert np.abs(out - z[f"stft/{name}"]).max() <= 1e-5


def test_torch_cpu_unet_matches_goldens_and_numpy_oracle():
    """oracle/unet_torch.py (the CPU baseline bench.py times) against the reference-generated
    forward goldens and the numpy oracle."""
    import torch
    from oracle import unet as ounet
    from oracle.unet_torch import UNetTorch
    from _helpers import golden, rms, unet_arch, unet_params
    torch.set_num_threads(4)
    fw = golden("unet_forward.npz")
    for N in (2112, 16448):
        net = UNetTorch(unet_params(N), unet_arch(N))
        got = net(fw[f"fw/{N}/cond"], fw[f"fw/{N}/x_t"], fw[f"fw/{N}/noise_level"])
        assert rms(got, fw[f"fw/{N}/eps"]) <= 1e-5
    N = 2112
    cond, x, nl = fw[f"fw/{N}/cond"], fw[f"fw/{N}/x_t"], fw[f"fw/{N}/noise_level"]
    ref = ounet.forward(unet_params(N), unet_arch(N), cond, x, nl)
    assert rms(UNetTorch(unet_params(N), unet_arch(N))(cond, x, nl), ref) <= 1e-5


# ---------------- the reference's own torch noise (SURVEY §8(b) noise_mode 1) ----------------
def test_oracle_with_reference_torch_noise():
    """torch_noise.npz: the reference run with torch.manual_seed(seed) and its own randn draws.
    model.model.reference_noise re-draws them in the reference's order (CPU generator); the oracle
    fed with them reproduces the reference output -- pins the draw order the HIP path replays."""
    import torch
    import model.diffusion as D
    import model.model as M
    import model.network as NW
    from _helpers import UNET_NET, parse_sched_key, tables_from_golden
    from oracle import schedule as osched
    z = golden("torch_noise.npz")
    for mode in ("condition_in", "supportive"):
        key = [k.rsplit("/", 1)[0] for k in z.files if k.startswith(f"torchnoise/unet/{mode}/") and k.endswith("/out")][0]
        sk = key.split("/")[3]
        N = int(key.split("/")[4].split("x")[0])
        sched = parse_sched_key(sk)
        m = M.SDDM(D.GaussianDiffusion(*sched, device="cpu"), NW.UNetModified2(num_samples=N, **UNET_NET["args"]),
                   p_transition=mode)
        cond = z[key + "/cond"]
        torch.manual_seed(int(z[key + "/seed"]))
        noise = M.reference_noise(m, torch.from_numpy(cond), device="cpu").numpy()
        P, arch = unet_params(N), unet_arch(N)
        tab = osched.make_tables(*sched)
        out = sampler.infer(lambda c, x, nl: unet.forward(P, arch, c, x, nl), tab, cond, mode=mode, noise=noise)
        assert rms(out, z[key + "/out"]) <= 1e-5, (mode, rms(out, z[key + "/out"]))
