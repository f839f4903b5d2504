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


_BENCH_ROWS = {}


def bench_rows(N=16448, B=16):
    """16 distinct rows of the bench shape: VoiceBank-shaped conditions, x_t drawn at 16 different
    noise levels of the headline schedule (linear 1e-6..1e-3, T=1000), and the numpy oracle's
    fp32 forward of every row (pinned to the reference goldens by tests/test_oracle.py)."""
    if (N, B) not in _BENCH_ROWS:
        from oracle import schedule as osched
        from oracle import unet as ounet
        from sddm_hip.synth import noisy_speech
        from _helpers import unet_arch
        tab = osched.make_tables("linear", 1000, 1e-6, 1e-3)
        ts = np.linspace(1000, 1, B).round().astype(int)
        nl = tab["sqrt_alpha_bar"][ts].astype(np.float32)
        cond = noisy_speech(B, N, seed=21)
        z = np.random.default_rng(22).standard_normal((B, 1, N)).astype(np.float32)
        x_t = (nl[:, None, None] * cond + np.sqrt(1 - nl[:, None, None] ** 2) * z).astype(np.float32)
        ref = ounet.forward(unet_params(N), unet_arch(N), cond, x_t, nl)
        _BENCH_ROWS[(N, B)] = (cond, x_t, nl, ref)
    return _BENCH_ROWS[(N, B)]


# per-layer kernel table exercising every kernel family on the bench geometry (tile configurations
# of 1, 2, 4, 6 and 8 waves, the 512-pixel tile, stride 2, upsample, virtual concat, res_conv chunks, conv_deep tiles)
_TUNING = {"downs.4": "tile:2", "downs.5.block1": "tile:10", "downs.5.block2": "tile:6", "downs.6": "tile:4",
           "downs.7.block1": "tile:8", "downs.8": "tile:7", "downs.9.block2": "deep:32:8", "downs.10": "tile:9",
           "mid.0.block1": "tile:8", "mid.0.block2": "deep", "ups.0.block1": "tile:9", "ups.4": "tile:6",
           "ups.5.block1": "tile:11", "ups.7": "tile:3", "ups.8.block1": "tile:1", "ups.8.block2": "tile:0",
           "ups.11.block1": "tile:1", "ups.12.block1": "strip", "downs.3.block2": "tile:12"}


# conv_deep with 16-channel blocks: every pixel tile (16..128), both wave counts, stride 2,
# upsample, virtual concat, identity residual and res_conv chunks
_TUNING16 = {"downs.7.block1": "deep:64:8:16", "downs.7.block2": "deep:128:4:16", "downs.8": "deep:32:4:16",
             "downs.9.block1": "deep:32:8:16", "downs.9.block2": "deep:16:4:16", "downs.10": "deep:16:4:16",
             "mid.0.block1": "deep:16:4:16", "mid.0.block2": "deep:32:4:16", "ups.0.block1": "deep:32:8:16",
             "ups.0.block2": "deep:16:4:16", "ups.1": "deep:64:4:16", "ups.4": "deep:128:8:16",
             "ups.5.block1": "deep:64:8:16", "ups.6.block2": "deep:128:4:16"}

# conv_deep with 64-channel blocks (the Cout = 128 layers): 4 and 8 waves, 32- and 64-pixel tiles,
# stride 2, upsample, virtual concat, identity residual and res_conv chunks
_TUNING64 = {"downs.7.block1": "deep:32:4:64", "downs.7.block2": "deep:64:4:64", "downs.8": "deep:32:4:64",
             "ups.2.block1": "deep:32:8:64", "ups.2.block2": "deep:64:4:64", "ups.3.block1": "deep:64:4:64",
             "ups.3.block2": "deep:32:4:64", "ups.4": "deep:64:4:64"}

# the bottom level (downs.10, mid.0, ups.0) as one launch (conv_chain.hip)
_CHAIN = {"downs.10": "chain", "mid.0.block1": "chain", "mid.0.block2": "chain", "ups.0.block1": "chain",
          "ups.0.block2": "chain"}

# producers of 32 tiles per image at 32x16 (16-pixel deep tiles): their consumers (downs.7.block2,
# ups.5.block2) combine 128 / 96 (tile, channel) statistics per group, more than one GroupNorm load
# round trip holds (64), so they take the fp64 two-pass finalize (gn_fused_prologue)
_TUNING16_GN = {**_TUNING16, "downs.7.block1": "deep:16:4:16", "ups.5.block1": "deep:16:4:16",
                "ups.5.block2": "deep:128:8:16"}


@pytest.mark.parametrize("dtype,tol,tuned", [("float32", 1e-4, None), ("bfloat16", 2.5e-2, None),
                                            ("bfloat16", 2.5e-2, "table"), ("bfloat16", 2.5e-2, "repo"),
                                            ("bfloat16", 2.5e-2, "table16"), ("float32", 1e-4, "table16"),
                                            ("bfloat16", 2.5e-2, "table16gn"), ("bfloat16", 2.5e-2, "table64"),
                                            ("float16", 5e-3, "table64"), ("bfloat16", 2.5e-2, "chain"),
                                            ("float16", 5e-3, "chain"), ("float16", 5e-3, None)])
def test_unet_forward_bench_batch(torch_cuda, dtype, tol, tuned):
    """B=16 x N=16448 (the bench shape), 16 distinct rows at 16 noise levels: the kernels and tiles
    picked for a full lane (and per-layer kernels set through sddm_set_conv_tuning: a table
    covering every kernel family, and the repository's measured table) reproduce the oracle on
    every row, so no row-offset / lane / per-row embedding error can hide behind identical rows."""
    import os
    N, B = 16448, 16
    cond, x_t, nl, ref = bench_rows(N, B)
    dev = torch_cuda.device("cuda", 0)
    ctx = make_ctx(N, dtype)
    if tuned in ("table", "table16", "table16gn", "table64", "chain"):
        # per-layer kernels everywhere
        ctx.set_conv_tuning({"lane_batch": B, "dtype": dtype, "num_samples": N,
                             "kernel": {"table": _TUNING, "table16": _TUNING16, "table16gn": _TUNING16_GN,
                                        "table64": _TUNING64, "chain": _CHAIN}[tuned]})
        ctx.profile(True)
    elif tuned == "repo":
        text, tab = repo_tuning_table(N, B)
        if tab is None:
            pytest.skip("no measured per-layer table in the repository")
        ctx.set_conv_tuning(text)
        ctx.profile(True)
    eps = torch_cuda.full((B, 1, N), float("nan"), device=dev)
    ctx.network_forward(torch_cuda.from_numpy(cond).to(dev), torch_cuda.from_numpy(x_t).to(dev),
                        torch_cuda.from_numpy(nl).to(dev), eps)
    torch_cuda.cuda.synchronize()
    if tuned == "repo":     # the headline table is the one the plan took (the file holds several)
        got = planned_kernels(ctx)
        ctx.profile(False)
        for layer, k in tab["kernel"].items():
            assert got.get(layer) == k, f"{layer}: table names {k}, plan ran {got.get(layer)}"
    elif tuned == "table16gn":   # the many-tile producers really ran (else the fallback went untested)
        got = planned_kernels(ctx)
        ctx.profile(False)
        for layer in ("downs.7.block1", "ups.5.block1", "downs.7.block2", "ups.5.block2"):
            assert got.get(layer) == _TUNING16_GN[layer], (layer, got.get(layer))
    elif tuned in ("table64", "chain"):     # every forced layer ran its kernel
        got = planned_kernels(ctx)
        ctx.profile(False)
        for layer, k in {"table64": _TUNING64, "chain": _CHAIN}[tuned].items():
            assert got.get(layer) == k, (layer, got.get(layer))
    eps = eps.cpu().numpy()
    errs = [rms(eps[b], ref[b]) for b in range(B)]
    print(f"{dtype} {tuned} B={B} forward: row rms min {min(errs):.3e} max {max(errs):.3e} (ref rms {rms(ref, 0):.3f})")
    assert np.isfinite(eps).all()
    assert max(errs) <= tol


@pytest.mark.parametrize("dtype,tol", [("bfloat16", 2.5e-2), ("float16", 5e-3)])
def test_unet_forward_reruns_bit_identical(torch_cuda, dtype, tol):
    """Every kernel reduces in a fixed order (no float atomics; the whole-K kernel's LDS-DMA staging
    and split-K reduction included): two calls on one plan and a call on a fresh context give the
    same bits, within the oracle tolerance, on 16 distinct bench rows."""
    N, B = 16448, 16
    cond, x_t, nl, ref = bench_rows(N, B)
    dev = torch_cuda.device("cuda", 0)
    outs = []
    for fresh in (0, 0, 1):
        if fresh or not outs:
            ctx = make_ctx(N, dtype)
        eps = torch_cuda.full((B, 1, N), float("nan"), device=dev)
        ctx.network_forward(torch_cuda.from_numpy(cond).to(dev), torch_cuda.from_numpy(x_t).to(dev),
                            torch_cuda.from_numpy(nl).to(dev), eps)
        torch_cuda.cuda.synchronize()
        outs.append(eps.cpu().numpy())
    errs = [rms(outs[0][b], ref[b]) for b in range(B)]
    print(f"{dtype} reruns: row rms vs oracle min {min(errs):.3e} max {max(errs):.3e}")
    assert np.isfinite(outs[0]).all() and max(errs) <= tol
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


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


def planned_kernels(ctx):
    """{layer: "strip" | "tile:<cfg>" | "deep:<mt>:<nw>:<nb>"} of the last profiled call (the
    tuning table's vocabulary, parsed from the profiled op names)."""
    got = {}
    for o in ctx.profile_ops():
        name, _, tag = o["name"].partition("[")
        if tag:
            tag = tag.rstrip("]")
            if tag == "chain":               # one launch for the bottom level's five convs
                for layer in name.split("+"):
                    got[layer] = "chain"
                continue
            got[name] = "strip" if tag == "strip" else (
                "tile:" + tag[4:] if tag.startswith("tile") else "deep:" + tag[4:].replace("_", ":"))
    return got


def repo_tuning_table(N, lane_batch):
    """(file text, the table for this geometry) of the repository's tuning file, or (None, None)."""
    import json
    import os
    path = os.path.join(os.path.dirname(sddm_hip.__file__), "..", "configs", "conv_tuning.json")
    if not os.path.exists(path):
        return None, None
    text = open(path).read()
    j = json.loads(text)
    tabs = [t for t in j.get("tables", [j]) if t["num_samples"] == N and t["lane_batch"] == lane_batch]
    return text, (tabs[0] if tabs else None)


@pytest.mark.parametrize("lane", [4, 8])
def test_unet_forward_small_lane_measured_table(torch_cuda, lane):
    """infer.py's batches (InferDataLoader batch_size 4: a few chunks per batch, reference
    infer.py:70-77) on lane_rows = 4 / 8 plans: the plan takes the repository's table measured for
    that lane batch (tools/gpu_tile_sweep.sh at --lane-rows 4 / 8), runs its kernel on every layer,
    and matches the oracle on distinct rows at distinct noise levels."""
    N = 16448
    cond, x_t, nl, ref = bench_rows(N, 16)
    cond, x_t, nl, ref = cond[:lane], x_t[:lane], nl[:lane], ref[:lane]
    text, tab = repo_tuning_table(N, lane)
    assert tab is not None, f"no measured table for lane batch {lane}"
    dev = torch_cuda.device("cuda", 0)
    cfg = unet_config(N, ("linear", 100, 1e-6, 1e-3))
    cfg["lane_rows"] = lane
    ctx = sddm_hip.Context(cfg, 0, "bfloat16")
    for k, v in unet_params(N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    ctx.set_conv_tuning(text)
    ctx.profile(True)
    eps = torch_cuda.full((lane, 1, N), float("nan"), device=dev)
    ctx.network_forward(torch_cuda.from_numpy(cond).to(dev), torch_cuda.from_numpy(x_t).to(dev),
                        torch_cuda.from_numpy(nl).to(dev), eps)
    torch_cuda.cuda.synchronize()
    got = planned_kernels(ctx)
    ctx.profile(False)
    for layer, k in tab["kernel"].items():
        assert got.get(layer) == k, f"{layer}: table names {k}, plan ran {got.get(layer)}"
    eps = eps.cpu().numpy()
    errs = [rms(eps[b], ref[b]) for b in range(lane)]
    print(f"lane_rows {lane} measured table: row rms max {max(errs):.3e}")
    assert np.isfinite(eps).all() and max(errs) <= 2.5e-2


_CONFIG5_ROWS = {}


def config5_rows():
    """4 rows of the config #5 chunk length (N=32832) at mixed noise levels and the numpy oracle's
    fp32 forward of them."""
    if not _CONFIG5_ROWS:
        from oracle import unet
        from sddm_hip.synth import noisy_speech
        from _helpers import unet_arch
        N, B = 32832, 4
        rng = np.random.default_rng(12)
        cond = noisy_speech(B, N, seed=12)
        x_t = (0.7 * cond + 0.7 * rng.standard_normal(cond.shape)).astype(np.float32)
        nl = np.array([0.99, 0.7, 0.4, 0.1], dtype=np.float32).reshape(B, 1, 1)
        _CONFIG5_ROWS["rows"] = (cond, x_t, nl, unet.forward(unet_params(N), unet_arch(N), cond, x_t, nl.reshape(-1)))
    return _CONFIG5_ROWS["rows"]


@pytest.mark.parametrize("dtype,tol", [("float32", 1e-4), ("float16", 5e-3)])
def test_unet_forward_config5_geometry(torch_cuda, dtype, tol):
    """BASELINE config #5 shape: 2.05 s chunks (N=32832, 512 frames; every level twice as tall)
    in fp16 storage with fp32 GroupNorm statistics, against the numpy oracle, B=4 with mixed
    noise levels (parity unpinned by a reference golden at this length: oracle only)."""
    N, B = 32832, 4
    cond, x_t, nl, ref = config5_rows()
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


def test_unet_forward_config5_measured_table(torch_cuda):
    """The repository's tuning file holds one table per measured geometry ({"tables": [...]}); a
    config #5 plan (64-row lanes, N=32832, fp16) takes the config #5 table -- every conv runs the
    kernel that table names, checked on the profiled op names -- and reproduces the oracle."""
    N, B = 32832, 4
    text, tab = repo_tuning_table(N, 64)
    if tab is None:
        pytest.skip("no config #5 table in the repository")
    want = tab["kernel"]
    cond, x_t, nl, ref = config5_rows()
    cfg = unet_config(N)
    cfg["lane_rows"] = 64
    ctx = sddm_hip.Context(cfg, 0, "float16")
    for k, v in unet_params(N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    ctx.set_conv_tuning(text)
    dev = torch_cuda.device("cuda", 0)
    eps = torch_cuda.full((B, 1, N), float("nan"), device=dev)
    ctx.profile(True)
    ctx.network_forward(torch_cuda.from_numpy(cond).to(dev), torch_cuda.from_numpy(x_t).to(dev),
                        torch_cuda.from_numpy(nl).to(dev), eps)
    torch_cuda.cuda.synchronize()
    got = planned_kernels(ctx)
    ctx.profile(False)
    for layer, k in want.items():
        assert got.get(layer) == k, f"{layer}: table names {k}, plan ran {got.get(layer)}"
    out = eps.cpu().numpy()
    assert np.isfinite(out).all()
    err = rms(out, ref)
    print(f"config #5 table, fp16 forward N={N}: rms err {err:.3e}")
    assert err <= 5e-3


def test_multilane_graph_replay_equals_row_blocks(torch_cuda, monkeypatch):
    """B=40 = three lanes of 16 rows (graph-replayed concurrently on three streams, each lane with
    its own step counter and row offset) equals separate calls on the row blocks, bit for bit;
    the non-graph path gives the same bits; 4-row lanes (10 lanes on 4 streams) equal their own
    row blocks and stay close to the 16-row-lane result."""
    from sddm_hip.synth import noisy_speech
    N, B, sched = 2112, 40, ("linear", 6, 1e-6, 1e-3)
    cond = noisy_speech(B, N, seed=77)
    monkeypatch.setenv("SDDM_LANE_ROWS", "16")
    ctx = make_ctx(N, "bfloat16", sched)
    full = _sample(torch_cuda, ctx, cond)
    blocks = np.concatenate([_sample(torch_cuda, ctx, cond[r:r + 16], row_offset=r) for r in (0, 16, 32)])
    assert np.isfinite(full).all()
    assert np.array_equal(full, blocks)
    monkeypatch.setenv("SDDM_NO_GRAPH", "1")
    assert np.array_equal(_sample(torch_cuda, make_ctx(N, "bfloat16", sched), cond), full)
    monkeypatch.delenv("SDDM_NO_GRAPH")
    monkeypatch.setenv("SDDM_LANE_ROWS", "64")
    full64 = _sample(torch_cuda, make_ctx(N, "bfloat16", sched), cond)   # one 40-row lane
    assert np.array_equal(full64, _sample(torch_cuda, make_ctx(N, "bfloat16", sched), cond))
    print(f"one 40-row lane vs 16-row lanes: rms {rms(full64, full):.3e}")
    assert rms(full64, full) <= 1e-2
    monkeypatch.setenv("SDDM_LANE_ROWS", "4")
    ctx4 = make_ctx(N, "bfloat16", sched)
    full4 = _sample(torch_cuda, ctx4, cond)
    blocks4 = np.concatenate([_sample(torch_cuda, ctx4, cond[r:r + 8], row_offset=r) for r in range(0, B, 8)])
    assert np.array_equal(full4, blocks4)
    err = rms(full4, full)
    print(f"4-row lanes vs 16-row lanes: rms {err:.3e}")
    assert err <= 1e-2


_HEADLINE32 = {}


@pytest.mark.parametrize("dtype,gate", [("bfloat16", 5e-3), ("float16", 1e-3)])
def test_headline_16bit_vs_fp32_1000_steps(torch_cuda, dtype, gate):
    """The benchmarked workload (config #2: T=1000, B=16 x 16448, linear 1e-6..1e-3, condition_in)
    sampled in 16 bits and in fp32 on the HIP path from the same seed: the RMS difference of the
    denoised outputs is the drift DESIGN.md §4 quotes (fp32 itself is pinned to the reference at
    <= 1.2e-7 RMS by the sampling-loop tests).  fp16 keeps the same bytes and MFMA rate as bf16 and
    stays inside north_star's 1e-3 bar; bf16 (the configured headline dtype) does not."""
    from sddm_hip.synth import noisy_speech
    N, B, sched = 16448, 16, ("linear", 1000, 1e-6, 1e-3)
    cond = noisy_speech(B, N, seed=1234)
    if "out" not in _HEADLINE32:
        _HEADLINE32["out"] = _sample(torch_cuda, make_ctx(N, "float32", sched), cond)
    out32 = _HEADLINE32["out"]
    out16 = _sample(torch_cuda, make_ctx(N, dtype, sched), cond)
    assert np.isfinite(out16).all() and np.isfinite(out32).all()
    err = rms(out16, out32)
    rows = [rms(out16[b], out32[b]) for b in range(B)]
    print(f"T=1000 B=16 {dtype} vs fp32: rms {err:.3e}, worst row {max(rows):.3e}, signal rms {rms(out32, 0):.3f}")
    assert err <= gate


def test_config5_sampling_b128_lanes(torch_cuda):
    """BASELINE config #5 per-GPU plan: B=128 chunks of 32832 samples in fp16 = 2 lanes of 64 rows
    (lane_rows = 64, as bench.py sets it for per-GPU batches of 64+) graph-replayed on 2 streams.  A 3-step sampling run equals separate
    64-row runs of its two row blocks (row_offset keyed noise) bit for bit, and stays within the
    fp16 sampling tolerance of the fp32 path (fp32 itself pinned to the reference goldens)."""
    from sddm_hip.synth import noisy_speech
    N, B, sched = 32832, 128, ("linear", 3, 1e-6, 1e-3)
    cond = noisy_speech(B, N, seed=55)
    cfg = unet_config(N, sched)
    cfg["lane_rows"] = 64
    ctx = sddm_hip.Context(cfg, 0, "float16")
    for k, v in unet_params(N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    full = _sample(torch_cuda, ctx, cond)
    assert np.isfinite(full).all()
    for r in (0, 64):
        assert np.array_equal(full[r:r + 64], _sample(torch_cuda, ctx, cond[r:r + 64], row_offset=r))
    ref = _sample(torch_cuda, make_ctx(N, "float32", sched), cond[112:128], row_offset=112)
    err = rms(full[112:128], ref)
    print(f"config #5 B=128 fp16 vs fp32 (rows 112..127, 3 steps): rms {err:.3e}")
    assert err <= 5e-3
