"""GPU parity of the HIP sampler against the golden vectors and the CPU oracle.

Everything here calls libsddm_hip.so through its C ABI (ctypes); no torch compute is used
except allocation and copies.  Tolerances:
  fp32 network forward       RMS <= 1e-4   (measured ~1e-6; reference fp32 vs fp64 is 1e-6)
  fp32 sampling loop         RMS <= 1e-3   (north_star parity bar)
  bf16 / fp16 network forward RMS <= 2.5e-2 / 5e-3 of an output RMS ~0.64 (reduced-precision storage)
  transitions                max |diff| <= 2e-6 (only the Box-Muller ulps differ)
"""
import numpy as np
import pytest

import sddm_hip
from _helpers import golden, parse_sched_key, rms, tables_from_golden, unet_config, unet_params

pytestmark = pytest.mark.gpu


def make_ctx(N, dtype="float32", sched=("linear", 100, 1e-6, 1e-3), mode="condition_in", tables=None):
    ctx = sddm_hip.Context(unet_config(N, sched, mode), 0, dtype)
    for k, v in unet_params(N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    if tables is not None:
        for k, v in tables.items():
            ctx.load_param("diffusion." + k, v)
    assert ctx.missing() == 0
    return ctx


def _forward(torch, ctx, fw, N):
    dev = torch.device("cuda", 0)
    cond = torch.from_numpy(fw[f"fw/{N}/cond"]).to(dev)
    x_t = torch.from_numpy(fw[f"fw/{N}/x_t"]).to(dev)
    nl = torch.from_numpy(fw[f"fw/{N}/noise_level"]).to(dev)
    eps = torch.full_like(cond, float("nan"))
    ctx.network_forward(cond, x_t, nl, eps)
    torch.cuda.synchronize()
    return eps.cpu().numpy()


@pytest.mark.parametrize("N", [2112, 16448])
def test_unet_forward_fp32_matches_reference(torch_cuda, N):
    fw = golden("unet_forward.npz")
    eps = _forward(torch_cuda, make_ctx(N), fw, N)
    ref = fw[f"fw/{N}/eps"]
    assert np.isfinite(eps).all()
    err = rms(eps, ref)
    print(f"fp32 forward N={N}: rms err {err:.3e} (ref rms {rms(ref, 0):.3f})")
    assert err <= 1e-4


@pytest.mark.parametrize("dtype,tol", [("bfloat16", 2.5e-2), ("float16", 5e-3)])
def test_unet_forward_reduced_precision(torch_cuda, dtype, tol):
    N = 2112
    fw = golden("unet_forward.npz")
    eps = _forward(torch_cuda, make_ctx(N, dtype), fw, N)
    err = rms(eps, fw[f"fw/{N}/eps"])
    print(f"{dtype} forward: rms err {err:.3e}")
    assert err <= tol


@pytest.mark.parametrize("dtype,tol,tuned", [("float32", 1e-4, False), ("bfloat16", 2.5e-2, False),
                                            ("bfloat16", 2.5e-2, True)])
def test_unet_forward_bench_batch(torch_cuda, dtype, tol, tuned):
    """B=16 x N=16448 (the bench shape): the kernel/tile configurations picked for a full batch
    (not the B=1 ones) -- and per-layer tiles set through sddm_set_conv_tuning -- reproduce the
    reference on every row; rows use mixed noise levels."""
    N, B = 16448, 16
    fw = golden("unet_forward.npz")
    dev = torch_cuda.device("cuda", 0)
    cond = np.repeat(fw[f"fw/{N}/cond"], B, axis=0)
    x_t = np.repeat(fw[f"fw/{N}/x_t"], B, axis=0)
    nl = np.repeat(fw[f"fw/{N}/noise_level"], B, axis=0)
    ctx = make_ctx(N, dtype)
    if tuned:     # sddm_set_conv_tuning: per-layer conv_deep tiles other than the heuristic's
        ctx.set_conv_tuning({"lane_batch": B, "dtype": dtype, "num_samples": N,
                             "deep": {"downs.6": [64, 4], "downs.8": [32, 8], "mid.0.block1": [32, 8],
                                      "ups.5.block1": [64, 4], "ups.7": [128, 4]}})
    eps = torch_cuda.full((B, 1, N), float("nan"), device=dev)
    ctx.network_forward(torch_cuda.from_numpy(cond).to(dev), torch_cuda.from_numpy(x_t).to(dev),
                        torch_cuda.from_numpy(nl).to(dev), eps)
    torch_cuda.cuda.synchronize()
    eps = eps.cpu().numpy()
    ref = fw[f"fw/{N}/eps"][0]
    errs = [rms(eps[b], ref) for b in range(B)]
    print(f"{dtype} B={B} forward: worst row rms {max(errs):.3e}")
    assert np.isfinite(eps).all()
    assert max(errs) <= tol


def _sample(torch, ctx, cond_np, seed=7, row_offset=0):
    dev = torch.device("cuda", 0)
    cond = torch.from_numpy(np.ascontiguousarray(cond_np)).to(dev)
    out = torch.full_like(cond, float("nan"))
    ctx.sample(cond, out, seed, row_offset)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _infer_keys():
    inf = golden("unet_infer.npz")
    return sorted({k.rsplit("/", 1)[0] for k in inf.files})


@pytest.mark.parametrize("key", _infer_keys())
def test_sampling_loop_fp32_matches_reference(torch_cuda, key):
    inf = golden("unet_infer.npz")
    _, mode, sk, shp = key.split("/")
    N, B = map(int, shp.split("x"))
    ctx = make_ctx(N, "float32", parse_sched_key(sk), mode, tables_from_golden(sk))
    out = _sample(torch_cuda, ctx, inf[key + "/cond"])
    ref = inf[key + "/out"]
    err = rms(out, ref)
    print(f"{key}: rms {err:.3e}")
    assert np.isfinite(out).all()
    assert err <= 1e-3


def test_sharded_rows_equal_single_run(torch_cuda):
    """Row blocks sampled with row_offset reproduce the same rows of one batch bit-exactly (§8e)."""
    from sddm_hip.synth import noisy_speech
    N = 2112
    cond = noisy_speech(4, N, seed=99)
    full = _sample(torch_cuda, make_ctx(N, "bfloat16", ("linear", 4, 1e-6, 1e-3)), cond)
    ctx = make_ctx(N, "bfloat16", ("linear", 4, 1e-6, 1e-3))
    a = _sample(torch_cuda, ctx, cond[:2], row_offset=0)
    b = _sample(torch_cuda, ctx, cond[2:], row_offset=2)
    assert np.array_equal(np.concatenate([a, b]), full)
    again = _sample(torch_cuda, ctx, cond[2:], row_offset=2)
    assert np.array_equal(again, b)  # deterministic (no atomics)


def test_transitions_match_reference(torch_cuda):
    tr = golden("transitions.npz")
    dev = torch_cuda.device("cuda", 0)
    keys = sorted({k.rsplit("/", 1)[0] for k in tr.files})
    worst = 0.0
    for key in keys:
        parts = key.split("/")
        sk, mode = parts[1], parts[2]
        ctx = sddm_hip.Context({"arch": {"type": "SDDM", "args": {}},
                                "diffusion": {"type": "GaussianDiffusion",
                                              "args": dict(zip(("schedule", "n_timestep", "linear_start",
                                                                "linear_end"), parse_sched_key(sk)))}})
        for k, v in tables_from_golden(sk).items():
            ctx.load_param("diffusion." + k, v)
        ref = tr[key + "/out"]
        out = torch_cuda.empty(ref.shape, dtype=torch_cuda.float32, device=dev)
        if mode.startswith("get_x_T"):
            cond = torch_cuda.from_numpy(tr[key + "/cond"]).to(dev)
            ctx.initial_state(sddm_hip.TR_CONDITION_IN if mode == "get_x_T" else sddm_hip.TR_CONDITIONAL,
                              cond, out, 7)
        else:
            t = int(parts[3])
            x_t, eps, cond = (torch_cuda.from_numpy(tr[key + f"/{n}"]).to(dev) for n in ("x_t", "eps", "cond"))
            ctx.transition(sddm_hip.TRANSITIONS[mode], x_t, eps, cond, t, out, 7)
        torch_cuda.cuda.synchronize()
        o = out.cpu().numpy()
        assert np.array_equal(np.isnan(o), np.isnan(ref)), key
        if not np.isnan(ref).all():
            d = float(np.nanmax(np.abs(o - ref)))
            worst = max(worst, d)
            assert d <= 2e-6, (key, d)
    print("worst transition diff", worst)


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-4), ("float16", 5e-3)])
def test_unet_forward_config5_geometry(torch_cuda, dtype, tol):
    """BASELINE config #5 shape: 2.05 s chunks (N=32832, 512 frames; every level twice as tall)
    in fp16 storage with fp32 GroupNorm statistics, against the numpy oracle, B=4 with mixed
    noise levels (parity unpinned by a reference golden at this length: oracle only)."""
    from oracle import unet
    from sddm_hip.synth import noisy_speech
    from _helpers import unet_arch
    N, B = 32832, 4
    rng = np.random.default_rng(12)
    cond = noisy_speech(B, N, seed=12)
    x_t = (0.7 * cond + 0.7 * rng.standard_normal(cond.shape)).astype(np.float32)
    nl = np.array([0.99, 0.7, 0.4, 0.1], dtype=np.float32).reshape(B, 1, 1)
    ref = unet.forward(unet_params(N), unet_arch(N), cond, x_t, nl.reshape(-1))
    dev = torch_cuda.device("cuda", 0)
    eps = torch_cuda.full((B, 1, N), float("nan"), device=dev)
    make_ctx(N, dtype).network_forward(torch_cuda.from_numpy(cond).to(dev), torch_cuda.from_numpy(x_t).to(dev),
                                       torch_cuda.from_numpy(nl).to(dev), eps)
    torch_cuda.cuda.synchronize()
    got = eps.cpu().numpy()
    assert np.isfinite(got).all()
    err = rms(got, ref)
    print(f"{dtype} forward N={N}: rms err {err:.3e}")
    assert err <= tol
