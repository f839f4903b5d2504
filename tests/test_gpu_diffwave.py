"""GPU: DiffWave (reference model/diffwave.py) and SDDM_spectrogram.infer (model.py:212-257)
through the facade and libsddm_hip, against goldens generated from the reference."""
import numpy as np
import pytest
import torch

from _helpers import diffwave_params, golden, parse_sched_key, rms

pytestmark = pytest.mark.gpu


def _net(dtype="float32"):
    import model.network as NW
    n = NW.DiffWave(num_samples=-1, num_timesteps=3, freq_bins=513, residual_channels=64, residual_layers=30,
                    dilation_cycle_length=10)
    n.load_state_dict({k: torch.from_numpy(v) for k, v in diffwave_params().items()})
    n.compute_dtype = dtype
    return n.cuda()


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-4), ("bfloat16", 3e-2), ("float16", 5e-3)])
def test_diffwave_forward_matches_reference(torch_cuda, dtype, tol):
    z = golden("diffwave.npz")
    k = "dw/fw/6x2"
    n = _net(dtype)
    spec, audio = (torch.from_numpy(z[f"{k}/{x}"]).cuda() for x in ("spec", "audio"))
    step = torch.from_numpy(z[f"{k}/step"]).reshape(-1, 1, 1).cuda()
    eps = n(spec, audio, step).cpu().numpy()
    ref = z[f"{k}/eps"]
    assert eps.shape == ref.shape
    assert rms(eps, ref) <= tol * max(1.0, float(np.sqrt(np.mean(ref ** 2))))


def test_sddm_spectrogram_infer_matches_reference(torch_cuda):
    import model.diffusion as D
    import model.model as M
    z = golden("diffwave.npz")
    sk = "linear_3_0.0001_0.05"
    k = f"dw/inf/time_step/{sk}/6x2"
    d = D.GaussianDiffusion(*parse_sched_key(sk), device="cuda")
    m = M.SDDM_spectrogram(d, _net(), hop_samples=256, noise_condition="time_step").cuda()
    out = m.infer(torch.from_numpy(z[f"{k}/spec"]).cuda(), seed=7).cpu().numpy()
    assert out.shape == z[f"{k}/out"].shape
    assert rms(out, z[f"{k}/out"]) <= 1e-3
    # continuous sampling records x_{t-1} after every step (T=3: inter 1)
    spec1 = torch.from_numpy(z[f"{k}/spec"][:1]).cuda()
    rec = m.infer(spec1, continuous=True, seed=7)
    assert len(rec) == 1 + 3
    got = np.stack([r.cpu().numpy() for r in rec[1:]])
    assert rms(got, z[f"{k}/steps"][:, :1]) <= 1e-3


def test_diffwave_rejects_bad_geometry(torch_cuda):
    n = _net()
    spec = torch.rand(1, 513, 2, device="cuda")
    with pytest.raises(Exception):
        n(spec, torch.zeros(1, 1, 500, device="cuda"), torch.ones(1, 1, 1, device="cuda"))


def test_diffwave_row_sharding_is_bit_identical(torch_cuda):
    """Rows sampled in two shards (row_offset) equal the rows of one batch."""
    import model.diffusion as D
    import model.model as M
    d = D.GaussianDiffusion("linear", 3, 1e-4, 0.05, device="cuda")
    m = M.SDDM_spectrogram(d, _net("bfloat16"), hop_samples=256, noise_condition="time_step",
                           compute_dtype="bfloat16").cuda()
    spec = torch.rand(4, 513, 4, generator=torch.Generator().manual_seed(2)).cuda()
    full = m.infer(spec, seed=5)
    a = m.infer(spec[:2].contiguous(), seed=5, row_offset=0)
    b = m.infer(spec[2:].contiguous(), seed=5, row_offset=2)
    assert torch.equal(full, torch.cat([a, b]))


def _dw_rows(B, F, seed):
    rng = np.random.default_rng(seed)
    spec = rng.uniform(0, 1, (B, 513, F)).astype(np.float32)          # U[0,1]
    audio = rng.standard_normal((B, 1, 256 * F)).astype(np.float32)
    steps = rng.integers(1, 201, B).astype(np.float32)              # time_step conditioning, T=200
    return spec, audio, steps


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-4), ("bfloat16", 3e-2)])
def test_diffwave_config3_geometry(torch_cuda, dtype, tol):
    """Config #3 geometry (config_diffwave.json: 63 frames x hop 256 = 16128 samples): 4 distinct
    rows at 4 diffusion steps against the numpy oracle -- covers the dilation <= 64 shared-window
    staging, the layer-major conditioner / z layouts and every partial tile of the layer kernel."""
    from oracle import diffwave as odw
    B, F = 4, 63
    spec, audio, steps = _dw_rows(B, F, 31)
    ref = odw.forward(diffwave_params(), spec, audio, steps)
    eps = _net(dtype)(torch.from_numpy(spec).cuda(), torch.from_numpy(audio).cuda(),
                      torch.from_numpy(steps).reshape(-1, 1, 1).cuda()).cpu().numpy()
    for b in range(B):
        err = rms(eps[b], ref[b])
        print(f"{dtype} row {b} step {steps[b]:.0f}: rms {err:.3e} (ref rms {rms(ref[b], 0):.3f})")
        assert err <= tol * max(1.0, rms(ref[b], 0))


def test_diffwave_config3_bench_batch(torch_cuda):
    """The benchmarked launch plan (B=64 x 63 frames, bf16) on 64 distinct rows; a spread of rows
    is checked against the oracle (a lane / row-offset error would show on these)."""
    from oracle import diffwave as odw
    B, F = 64, 63
    spec, audio, steps = _dw_rows(B, F, 32)
    eps = _net("bfloat16")(torch.from_numpy(spec).cuda(), torch.from_numpy(audio).cuda(),
                           torch.from_numpy(steps).reshape(-1, 1, 1).cuda()).cpu().numpy()
    assert np.isfinite(eps).all()
    rows = [0, 21, 42, 63]
    ref = odw.forward(diffwave_params(), spec[rows], audio[rows], steps[rows])
    for i, b in enumerate(rows):
        err = rms(eps[b], ref[i])
        print(f"bf16 B=64 row {b}: rms {err:.3e}")
        assert err <= 3e-2 * max(1.0, rms(ref[i], 0))


@pytest.mark.parametrize("dtype,tol", [("bfloat16", 3e-2), ("float16", 5e-3)])
@pytest.mark.parametrize("F", [1, 2, 5])
def test_diffwave_short_clips_dilation_chains(torch_cuda, dtype, tol, F):
    """Clips of 1 / 2 / 5 frames (256 / 512 / 1280 samples = 2 / 4 / 10 tiles of 128): the
    dilation-chain layers (d = 128 .. 512, dw_layer_chain_kernel) then have fewer tiles per clip
    than chains (d / 128), one-tile chains whose -d / +d tap images lie wholly outside the clip,
    and chains of uneven length; every row against the numpy oracle."""
    from oracle import diffwave as odw
    B = 3
    spec, audio, steps = _dw_rows(B, F, 40 + F)
    ref = odw.forward(diffwave_params(), spec, audio, steps)
    eps = _net(dtype)(torch.from_numpy(spec).cuda(), torch.from_numpy(audio).cuda(),
                      torch.from_numpy(steps).reshape(-1, 1, 1).cuda()).cpu().numpy()
    for b in range(B):
        err = rms(eps[b], ref[b])
        print(f"{dtype} F={F} row {b}: rms {err:.3e} (ref rms {rms(ref[b], 0):.3f})")
        assert np.isfinite(eps[b]).all() and err <= tol * max(1.0, rms(ref[b], 0))


def test_spectrogram_bin_count_is_checked(torch_cuda):
    """An 80-bin mel condition for a 513-bin DiffWave raises (the reference's Conv1d(freq_bins, ...)
    rejects it) instead of being read out of bounds by the library."""
    import model.diffusion as D
    import model.model as M
    n = _net()
    spec = torch.rand(1, 80, 2, device="cuda")
    with pytest.raises(RuntimeError):
        n(spec, torch.zeros(1, 1, 512, device="cuda"), torch.ones(1, 1, 1, device="cuda"))
    d = D.GaussianDiffusion("linear", 3, 1e-4, 0.05, device="cuda")
    m = M.SDDM_spectrogram(d, n, hop_samples=256, noise_condition="time_step").cuda()
    with pytest.raises(RuntimeError):
        m.infer(spec, seed=1)


def test_sddm_spectrogram_training_forward(torch_cuda):
    """SDDM_spectrogram inherits SDDM.forward (model.py:29-48): q-sample on HIP, then DiffWave on HIP
    with the time_step noise condition (level = t + r, continuous: diffwave.py:41-45 has no lookup),
    against oracle q_stochastic composed with oracle/diffwave.forward."""
    import model.diffusion as D
    import model.model as M
    from oracle import diffwave as odw, sampler as osamp
    from oracle.schedule import BUFFER_NAMES
    z = golden("diffwave.npz")
    k = "dw/fw/6x2"
    spec = z[f"{k}/spec"]
    B, N = spec.shape[0], 256 * spec.shape[-1]
    d = D.GaussianDiffusion("linear", 50, 1e-4, 0.05, device="cuda")
    m = M.SDDM_spectrogram(d, _net(), hop_samples=256, noise_condition="time_step").cuda()
    rng = np.random.default_rng(8)
    target = (0.3 * rng.standard_normal((B, 1, N))).astype(np.float32)
    noise = rng.standard_normal((B, 1, N)).astype(np.float32)
    t = np.array([3, 41], dtype=np.int64)[:B]
    r = rng.random(B).astype(np.float32)
    tg = lambda a: torch.from_numpy(a).cuda()
    with torch.no_grad():
        pred, nz = m(tg(target), tg(spec), noise=tg(noise), t=tg(t), random_step=tg(r))
    tab = {n: getattr(d, n).cpu().numpy() for n in BUFFER_NAMES}
    x_t, _, level = osamp.q_stochastic(tab, target, noise, t, r)
    ref = odw.forward(diffwave_params(), spec, x_t, np.asarray(level, np.float32).reshape(-1))
    assert pred.shape == (B, 1, N) and np.array_equal(nz.cpu().numpy(), noise)
    assert rms(pred.cpu().numpy(), ref) <= 1e-4 * max(1.0, float(np.sqrt(np.mean(ref.astype(np.float64) ** 2))))
