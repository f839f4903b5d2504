"""GPU: WaveGrad (reference model/wavegrad.py) and SDDM_spectrogram.infer (model.py:212-257, with the
SURVEY Q4 adapter) through the facade and libsddm_hip, against goldens generated from the reference
and the numpy oracle."""
import numpy as np
import pytest
import torch

from _helpers import golden, parse_sched_key, rms, wavegrad_params

pytestmark = pytest.mark.gpu


def _net(dtype="float32"):
    import model.network as NW
    n = NW.WaveGrad()
    n.load_state_dict({k: torch.from_numpy(v) for k, v in wavegrad_params().items()})
    n.compute_dtype = dtype
    return n.cuda()


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-4), ("bfloat16", 3e-2), ("float16", 5e-3)])
def test_wavegrad_forward_matches_reference(torch_cuda, dtype, tol):
    z = golden("wavegrad.npz")
    k = "wg/fw/6x2"
    n = _net(dtype)
    spec, audio, nl = (torch.from_numpy(z[f"{k}/{x}"]).cuda() for x in ("spec", "audio", "noise_level"))
    eps = n(spec, audio, nl).cpu().numpy()
    ref = z[f"{k}/eps"]
    assert eps.shape == ref.shape
    assert rms(eps, ref) <= tol * max(1.0, float(np.sqrt(np.mean(ref ** 2))))


def test_wavegrad_forward_matches_oracle_longer_clip(torch_cuda):
    """Every tile-boundary case of the conv kernel (lengths 16200..54, partial 128-sample tiles)."""
    from oracle import wavegrad as wg
    P = wavegrad_params()
    rng = np.random.default_rng(3)
    B, F = 3, 54
    spec = rng.uniform(0, 1, (B, 128, F)).astype(np.float32)
    audio = rng.standard_normal((B, 300 * F)).astype(np.float32)
    nl = np.array([0.9, 0.5, 0.1], dtype=np.float32)
    ref = wg.forward(P, spec, audio, nl)
    eps = _net()(*(torch.from_numpy(x).cuda() for x in (spec, audio, nl))).cpu().numpy()
    assert rms(eps, ref) <= 1e-4 * max(1.0, float(np.sqrt(np.mean(ref ** 2))))


def test_wavegrad_sampling_matches_reference(torch_cuda):
    import model.diffusion as D
    import model.model as M
    z = golden("wavegrad.npz")
    sk = "linear_3_0.0001_0.05"
    k = f"wg/inf/sqrt_alpha_bar/{sk}/6x2"
    d = D.GaussianDiffusion(*parse_sched_key(sk), device="cuda")
    m = M.SDDM_spectrogram(d, _net(), hop_samples=300).cuda()
    out = m.infer(torch.from_numpy(z[f"{k}/spec"]).cuda(), seed=7).cpu().numpy()
    assert out.shape == z[f"{k}/out"].shape
    assert rms(out, z[f"{k}/out"]) <= 1e-3
    spec1 = torch.from_numpy(z[f"{k}/spec"][:1]).cuda()
    rec = m.infer(spec1, continuous=True, seed=7)
    assert len(rec) == 1 + 3
    got = np.stack([r.cpu().numpy() for r in rec[1:]])
    assert rms(got, z[f"{k}/steps"][:, :1]) <= 1e-3


def test_wavegrad_row_sharding_is_bit_identical(torch_cuda):
    """Rows sampled in two shards (row_offset) equal the rows of one batch."""
    import model.diffusion as D
    import model.model as M
    d = D.GaussianDiffusion("linear", 3, 1e-4, 0.05, device="cuda")
    m = M.SDDM_spectrogram(d, _net("bfloat16"), hop_samples=300, compute_dtype="bfloat16").cuda()
    spec = torch.rand(4, 128, 6, generator=torch.Generator().manual_seed(1)).cuda()
    full = m.infer(spec, seed=11)
    a = m.infer(spec[:2].contiguous(), seed=11, row_offset=0)
    b = m.infer(spec[2:].contiguous(), seed=11, row_offset=2)
    assert torch.equal(full, torch.cat([a, b]))


def test_wavegrad_rejects_bad_geometry(torch_cuda):
    n = _net()
    spec = torch.rand(1, 128, 2, device="cuda")
    with pytest.raises(Exception):
        n(spec, torch.zeros(1, 500, device="cuda"), torch.ones(1, device="cuda"))


def test_wavegrad_single_clip_squeezes_like_reference(torch_cuda):
    """wavegrad.py:179 returns torch.squeeze(output): a single clip comes back as [N]."""
    from oracle import wavegrad as wg
    rng = np.random.default_rng(4)
    spec = rng.uniform(0, 1, (1, 128, 3)).astype(np.float32)
    audio = rng.standard_normal((1, 900)).astype(np.float32)
    nl = np.array([0.5], dtype=np.float32)
    out = _net()(*(torch.from_numpy(x).cuda() for x in (spec, audio, nl)))
    assert tuple(out.shape) == (900,)
    ref = wg.forward(wavegrad_params(), spec, audio, nl)[0]
    assert rms(out.cpu().numpy(), ref) <= 1e-4 * max(1.0, float(np.sqrt(np.mean(ref ** 2))))


def test_wavegrad_bf16_bench_batch(torch_cuda):
    """Config #4 per-GPU shape (B=64 x 54 frames x hop 300, bf16, the LDS-tiled conv plan) on 64
    distinct rows; a spread of rows is checked against the numpy oracle."""
    from oracle import wavegrad as wg
    B, F = 64, 54
    rng = np.random.default_rng(41)
    spec = rng.uniform(0, 1, (B, 128, F)).astype(np.float32)
    audio = rng.standard_normal((B, 300 * F)).astype(np.float32)
    nl = rng.uniform(0.05, 0.99, B).astype(np.float32)
    eps = _net("bfloat16")(*(torch.from_numpy(x).cuda() for x in (spec, audio, nl))).cpu().numpy()
    assert np.isfinite(eps).all()
    rows = [0, 19, 44, 63]
    ref = wg.forward(wavegrad_params(), spec[rows], audio[rows], nl[rows])
    for i, b in enumerate(rows):
        err = rms(eps[b], ref[i])
        print(f"bf16 B=64 row {b}: rms {err:.3e} (ref rms {rms(ref[i], 0):.3f})")
        assert err <= 3e-2 * max(1.0, rms(ref[i], 0))


def test_wavegrad_spectrogram_bin_count_is_checked(torch_cuda):
    n = _net()
    with pytest.raises(RuntimeError):
        n(torch.rand(1, 80, 2, device="cuda"), torch.zeros(1, 600, device="cuda"), torch.ones(1, device="cuda"))
