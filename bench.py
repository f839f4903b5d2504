#!/usr/bin/env python
"""Bench: denoised-audio seconds per second of 1000-step reverse diffusion with UNetModified2
(BASELINE.json metric; config_unet.json network, linear 1e-6..1e-3 schedule at T=1000).

One bench *step* = one full SDDM.infer sampling run (x_T -> x_0, T UNet evaluations + T
transitions) of a per-GPU batch of B synthetic 16 kHz chunks (16448 samples = 256 frames), entered
through the drop-in facade (model.model.SDDM.infer -> libsddm_hip).  With N GPUs every rank samples
its own B rows (row_offset = rank * B, so results equal a single-GPU run of all rows) and the
outputs are all-gathered over RCCL at the end of the step (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--timesteps T] [--dtype bf16]
    python bench.py --workload diffwave|wavegrad     # BASELINE configs #3 / #4 (not the headline)

At N=1 the headline line also carries `variants`: the fp32 parity path (2 timed runs) and the other
16-bit type (fp16 beside the bf16 headline, 5 timed runs), timed in the same process on the same
workload after the headline's timed region, each with the RMS drift of its output from the fp32
output of the same seed (`drift_vs_f32_rms`; north_star's bar is 1e-3).

Rank 0 prints one JSON line.  `roofline` is the dominant kernel's (the template instantiation with
the most time in a sampling run): algorithmic bytes per launch over its average duration, from HIP
events around every launch of one extra (untimed) sampling run, with the whole reverse step
reported beside it; `cpu_baseline` times a PyTorch-CPU restatement of the reference
(oracle/unet_torch.py) at the config's batch on this host's cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "speech-denoising-diffusion-model-2_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f16": 2500.0, "f32": 157.3}


def cpu_info():
    """CPU model name and core counts of this host (the run log records them)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return model, os.cpu_count() or 1, affinity


def cpu_baseline(B_cpu, k_steps, N, T):
    """SURVEY §8d CPU baseline: the reference's algorithm in PyTorch CPU ops (oracle/unet_torch.py,
    pinned to the reference goldens; tests-only restatement) at the config's batch, k reverse
    steps timed with torch.set_num_threads(os.cpu_count()), extrapolated x T/k (every step runs
    the same network; only t > 1 adds noise)."""
    sys.path.insert(0, REPO)
    import numpy as np
    import torch
    from oracle import philox, sampler, schedule, unet
    from oracle.unet_torch import UNetTorch
    from sddm_hip.synth import noisy_speech
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _weights import make_params, unet_shapes
    # the host cores this process may use: OMP_NUM_THREADS where the pool sets it (the GPU box caps a
    # job's CPU share with a quota while os.cpu_count() shows the whole machine; more threads than
    # the quota only oversubscribe it), else every core os.cpu_count() reports
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    torch.set_num_threads(threads)
    arch = unet.architecture(N, inner_channel=32, channel_mults=(1, 2, 3, 4, 5), res_blocks=1)
    net = UNetTorch(make_params(unet_shapes(arch), 0), arch)
    tab = schedule.make_tables("linear", T, 1e-6, 1e-3)
    cond = noisy_speech(B_cpu, N, seed=1234)
    x = sampler.get_x_T(tab, cond, philox.normal(7, 0, cond.shape))
    net(cond, x, np.full(B_cpu, tab["sqrt_alpha_bar"][T], np.float32))                  # warm-up
    t0 = time.perf_counter()
    for i in range(k_steps):
        t = T - i
        log(f"CPU step {i + 1}/{k_steps} ({threads} threads)")
        eps = net(cond, x, np.full(B_cpu, tab["sqrt_alpha_bar"][t], np.float32))
        x = sampler.transition("condition_in", tab, x, t, eps, cond, philox.normal(7, t, x.shape))
    dt = (time.perf_counter() - t0) / k_steps
    # a second timing at 8 threads (the survey's reference measurement used 8 Xeon threads): on a
    # shared host the job's CPU quota, not the core count, limits the wider run
    dt8 = None
    if threads != 8:
        torch.set_num_threads(8)
        log("CPU step at 8 threads")
        t1 = time.perf_counter()
        net(cond, x, np.full(B_cpu, tab["sqrt_alpha_bar"][T - k_steps], np.float32))
        dt8 = time.perf_counter() - t1
        torch.set_num_threads(threads)
    return B_cpu * N / 16000.0 / (dt * T), dt, threads, dt8


def cpu_quota():
    """The CPU share the host grants this job (cgroup v2 cpu.max: quota / period), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def init_ranks():
    """One process per GPU (torchrun env): bind this rank's device FIRST, then join the process
    group with that device (RCCL over xGMI creates its communicator on it).  SDDM_DIST_BACKEND=gloo
    rehearses the multi-rank path with several ranks sharing one GPU (RCCL refuses two ranks on one
    device); ranks wrap onto the visible devices."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local_dev = local_rank % max(ndev, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        backend = os.environ.get("SDDM_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
    return world, rank, dev


def log(msg):
    """progress on stderr (the JSON line stays the only stdout output)"""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def kernel_src_hash():
    """Hash of everything that decides which kernel runs each layer and how: the HIP sources, the
    runtime that plans the layers (sddm_runtime.cpp: choose_conv / choose_tile / choose_deep) and the
    measured per-layer kernel table (configs/conv_tuning.json).  A committed PMC traffic summary is
    used only for the kernels and layer plan it measured."""
    import glob
    import hashlib
    h = hashlib.sha256()
    # (the spectrogram samplers' sources are left out: they run none of the UNet's kernels)
    other = {"diffwave.hip", "dw_runtime.h", "wavegrad.hip", "wg_kernels.h", "wg_runtime.h", "stft.hip", "stft_kernels.h"}
    files = sorted(f for f in glob.glob(os.path.join(PKG, "csrc", "*.hip")) + glob.glob(os.path.join(PKG, "csrc", "*.h"))
                   if os.path.basename(f) not in other)
    files += [os.path.join(PKG, "csrc", "sddm_runtime.cpp"), os.path.join(PKG, "configs", "conv_tuning.json")]
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


TRAFFIC_FILES = ("r06_hbm_traffic.json", "r06_f16_hbm_traffic.json", "r06_config5_hbm_traffic.json",
                 "r05_hbm_traffic.json", "r05_config5_hbm_traffic.json", "r04_hbm_traffic.json",
                 "r04_config5_hbm_traffic.json")   # newest first


def unet_roofline(model, cond, N, B, T, dtype, ms_per_run):
    """Roofline of the dominant kernel (the template instantiation with the most time in one sampling
    run): algorithmic bytes per launch / its average launch duration, from HIP events recorded on the
    sampling stream around every launch of one extra (untimed, non-graph) sampling run of the same
    workload, all T steps.  The whole reverse step is reported beside it against the graph-replayed
    wall time of the timed region.  `traffic` (PMC HBM bytes per launch) comes from the committed
    rocprofv3 summary only when it was measured for this kernel, workload and kernel sources."""
    import torch
    ctx = model._context(cond.device)
    ctx.profile(True)
    model.infer(cond, seed=7)
    torch.cuda.synchronize()
    ops = ctx.profile_ops()
    ctx.profile(False)
    agg = {}
    for o in ops:
        a = agg.setdefault(o["kernel"], {"ms": 0.0, "n": 0, "bytes": 0.0, "flops": 0.0, "layers": []})
        a["ms"] += o["avg_ms"] * o["launches"]
        a["n"] += o["launches"]
        a["bytes"] += o["bytes"] * o["launches"]
        a["flops"] += o["flops"] * o["launches"]
        a["layers"].append(o["name"])
    total_ms = sum(a["ms"] for a in agg.values())
    dom = max(agg, key=lambda k: agg[k]["ms"])
    d = agg[dom]
    avg_ms, bpl, fpl = d["ms"] / d["n"], d["bytes"] / d["n"], d["flops"] / d["n"]
    gbs, tfs = bpl / (avg_ms * 1e-3) / 1e9, fpl / (avg_ms * 1e-3) / 1e12
    step_bytes, step_flops = sum(o["bytes"] for o in ops), sum(o["flops"] for o in ops)
    step_ms = ms_per_run / T
    traffic, tsrc = None, None
    key = {"N": N, "B": B, "dtype": dtype, "src": kernel_src_hash()}
    for name in TRAFFIC_FILES:
        tf = os.path.join(REPO, "profiles", name)
        if not os.path.exists(tf):
            continue
        with open(tf) as fh:
            pmc = json.load(fh)
        if all(pmc.get(k) == v for k, v in key.items()) and dom in pmc.get("kernels", {}):
            traffic = round(pmc["kernels"][dom]["bytes_per_launch"])
            tsrc = (f"profiles/{name} (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, same kernel sources, "
                    f"layer plan and workload)")
            break
    # the top single template instantiation (the family above merges e.g. the strip kernel's
    # residual-mode / GroupNorm variants, which rocprofv3 lists separately)
    inst = {}
    for o in ops:
        a = inst.setdefault(o.get("inst") or o["kernel"], {"ms": 0.0, "n": 0, "bytes": 0.0, "layers": []})
        a["ms"] += o["avg_ms"] * o["launches"]
        a["n"] += o["launches"]
        a["bytes"] += o["bytes"] * o["launches"]
        a["layers"].append(o["name"])
    top = max(inst, key=lambda k: inst[k]["ms"])
    ti = inst[top]
    ti_ms, ti_b = ti["ms"] / ti["n"], ti["bytes"] / ti["n"]
    ti_gbs = ti_b / (ti_ms * 1e-3) / 1e9
    top_inst = {"kernel": top, "layers": ti["layers"], "avg_launch_ms": round(ti_ms, 5),
                "alg_bytes_per_launch": round(ti_b), "achieved": round(ti_gbs, 1),
                "frac": round(ti_gbs / HBM_PEAK_GBS, 4), "share_of_launch_time": round(ti["ms"] / total_ms, 4)}
    fam = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4)}
    if dtype == "f32":
        # the fp32 UNet (82.8 FLOP/B against an fp32 ridge of ~20) is MFMA-fp32 bound
        fam = {"bound": "mfma", "achieved": round(tfs, 2), "peak": MFMA_PEAK_TFLOPS[dtype], "unit": "TFLOP/s",
               "frac": round(tfs / MFMA_PEAK_TFLOPS[dtype], 4), "hbm_gbs": round(gbs, 1),
               "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
    return {**fam, "traffic": traffic, "traffic_source": tsrc,
            "kernel": dom, "layers": d["layers"], "avg_launch_ms": round(avg_ms, 5), "launches_timed": d["n"],
            "share_of_launch_time": round(d["ms"] / total_ms, 4), "alg_bytes_per_launch": round(bpl),
            "mfma_tflops": round(tfs, 2), "mfma_frac": round(tfs / MFMA_PEAK_TFLOPS[dtype], 4),
            "top_instantiation": top_inst,
            "step": {"alg_bytes": round(step_bytes), "alg_flops": round(step_flops), "ms": round(step_ms, 5),
                     "achieved_gbs": round(step_bytes / (step_ms * 1e-3) / 1e9, 1),
                     "frac": round(step_bytes / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "mfma_tflops": round(step_flops / (step_ms * 1e-3) / 1e12, 2),
                     "launches": len(ops), "launch_time_ms": round(total_ms / T, 5)}}


DTYPE_NAMES = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}


def rms(a, b):
    """RMS difference of two sampled batches (tests/_helpers.py rms: the drift DESIGN.md §4 quotes)"""
    import torch
    return float(torch.sqrt(torch.mean((a.double() - b.double()) ** 2)).item())


def unet_variant(model, step, result, dtype, steps, warmup, N, B, T, cond_all, no_profile):
    """A precision sub-record of the headline line, timed in the same process on the same workload
    (same condition, seed and weights; the library packs the weights in `dtype`): W untimed runs, K
    timed runs bracketed by torch.cuda.synchronize(), the same roofline fields as the headline."""
    import torch
    model.compute_dtype = DTYPE_NAMES[dtype]
    log(f"{dtype} sub-record: {warmup} warmup + {steps} timed sampling runs")
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = result["out"].clone()
    if not torch.isfinite(out).all():
        raise RuntimeError(f"non-finite samples ({dtype})")
    v = {"value": round(steps * B * N / 16000.0 / el, 4), "unit": "audio_s/s", "steps": steps, "warmup": warmup,
         "ms_per_step": round(1e3 * el / steps, 3), "dtype": dtype}
    if not no_profile:
        v["roofline"] = unet_roofline(model, cond_all[:B].contiguous(), N, B, T, dtype, 1e3 * el / steps)
    v["out"] = out
    return v


# spectrogram-conditioned workloads (BASELINE.json configs #3 and #4): config, frames, clips per GPU,
# step-variant GFLOP per clip and step
# (SURVEY.md §8a rows a20 / a22, §8d): step-variant GFLOP and conv-boundary elements per clip and
# step, step-invariant elements per clip and sampling run (DiffWave's conditioner + upsampler)
SPEC_WORKLOADS = {
    "diffwave": dict(config="config_diffwave_bench.json", frames=63, batch=64, bins=513, gflop=31.85,
                     melems=220.9, inv_melems=319.5, bound="hbm",
                     label="DiffWave config_diffwave.json, linear 1e-4..0.02, T={T}, time_step conditioning"),
    "wavegrad": dict(config="config_wavegrad_bench.json", frames=54, batch=64, bins=128, gflop=47.38,
                     melems=92.8, inv_melems=0.0, bound="mfma",
                     label="WaveGrad, linear 1e-4..0.05, T={T} (SURVEY §8d fast schedule: T=50), sqrt_alpha_bar"),
}


def cpu_baseline_spec(workload, model, spec_np, T):
    """numpy oracle forward of one clip for one step (os.cpu_count() BLAS threads, set before numpy
    is first imported by the caller's environment), extrapolated x T (tests-only restatement)."""
    sys.path.insert(0, REPO)
    import numpy as np
    net = model.noise_estimate_model
    P = {k: v.detach().float().cpu().numpy() for k, v in net.state_dict().items()}
    spec = spec_np[:1]
    if workload == "diffwave":
        from oracle import diffwave as ora
        x = np.zeros((1, 1, 256 * spec.shape[-1]), np.float32)
        fn = lambda: ora.forward(P, spec, x, np.array([float(T)], np.float32))   # noqa: E731
    else:
        from oracle import wavegrad as ora
        x = np.zeros((1, 300 * spec.shape[-1]), np.float32)
        fn = lambda: ora.forward(P, spec, x, np.array([0.5], np.float32))       # noqa: E731
    fn()                                                                          # warm BLAS
    t0, reps = time.perf_counter(), 0
    while reps < 1 or time.perf_counter() - t0 < 10.0:                            # ~10 s of host work
        fn()
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    return x.size / 16000.0 / (dt * T), dt, reps


def main_spec(args):
    """SDDM_spectrogram.infer benches (DiffWave / WaveGrad), same contract as the UNet headline."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.network as module_network
    import model.model as module_arch

    W = SPEC_WORKLOADS[args.workload]
    world, rank, dev = init_ranks()
    cfg = read_json(os.path.join(PKG, "configs", W["config"]))
    if args.timesteps_set:
        cfg["diffusion"]["args"]["n_timestep"] = args.timesteps
    config = ConfigParser(cfg)
    T = cfg["diffusion"]["args"]["n_timestep"]
    B = args.batch if args.batch_set else W["batch"]
    F = W["frames"]
    hop = cfg["spectrogram"]["hop_samples"]
    N = hop * F
    torch.manual_seed(0)                                            # random-init weights
    # the reference config resolves as is (model.build_from_config: SURVEY Q5 / Q6)
    diffusion, network, model = module_arch.build_from_config(config, module_diffusion, module_network,
                                                              module_arch, dev)
    if args.workload == "diffwave":                                 # output_projection is zero-init
        with torch.no_grad():
            network.output_projection.weight.uniform_(-0.1, 0.1)
    model = model.to(dev).eval()
    model.compute_dtype = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}[args.dtype]
    rng = np.random.default_rng(1234)
    spec_all = rng.uniform(0, 1, (B * world, W["bins"], F)).astype(np.float32)   # U[0,1]
    spec = torch.from_numpy(spec_all).to(dev)
    result = {}

    def step():        # the product multi-GPU path: row shards + one RCCL all-gather
        result["out"] = module_arch.sharded_infer(model, spec, seed=7)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() != "gloo" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if not torch.isfinite(result["out"]).all():
        raise RuntimeError("non-finite samples")
    if rank == 0:
        es = 2 if args.dtype != "f32" else 4
        tfs = args.steps * T * B * W["gflop"] / elapsed / 1e3      # whole-job MFMA rate per GPU
        gbs = args.steps * B * (T * W["melems"] + W["inv_melems"]) * 1e6 * es / elapsed / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:             # CPU baseline: rank 0 at N=1 only
            v, dt, reps = cpu_baseline_spec(args.workload, model, spec_all, T)
            cpu_model, ncpu, naff = cpu_info()
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or ncpu
            cpu = {"value": round(v, 6), "unit": "audio_s/s", "cores": threads, "kind": "port",
                   "cpu_model": cpu_model, "cpu_count": ncpu, "cpu_affinity": naff,
                   "sample": f"numpy oracle, {reps} network evaluations of 1 clip ({dt:.2f} s each), "
                             f"extrapolated x{T} steps"}
        audio_s = args.steps * B * world * N / 16000.0
        line = {"metric": f"denoised audio sec/sec, {T}-step {network.__class__.__name__} @16kHz",
                "value": round(audio_s / elapsed, 4), "unit": "audio_s/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                "data": "synthetic spectrograms U[0,1], random-init weights",
                "config": {"workload": f"{W['label'].format(T=T)}, {B}x{N}-sample clips per GPU",
                           "model": network.__class__.__name__, "global_batch": B * world, "seq_len": N,
                           "timesteps": T, "parallelism": f"dp{world}"},
                "roofline": ({"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                              "kernel": "whole sampling run: SURVEY 8d conv-boundary bytes "
                                        f"({W['melems']} M elements/clip/step + {W['inv_melems']} M once) / wall",
                              "mfma_tflops": round(tfs, 2), "mfma_frac": round(tfs / MFMA_PEAK_TFLOPS[args.dtype], 4)}
                             if W["bound"] == "hbm" else
                             {"bound": "mfma", "achieved": round(tfs, 2), "peak": MFMA_PEAK_TFLOPS[args.dtype],
                              "unit": "TFLOP/s", "frac": round(tfs / MFMA_PEAK_TFLOPS[args.dtype], 4), "traffic": None,
                              "kernel": "whole sampling run (step-variant algorithmic FLOPs / wall)",
                              "hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}),
                "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16, help="clips per GPU")
    ap.add_argument("--timesteps", type=int, default=1000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3, help="CPU reverse steps at the config's batch (extrapolated x T)")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-variants", action="store_true", help="skip the same-run fp16 / fp32 sub-records")
    ap.add_argument("--lane-rows", type=int, default=None, help="rows per UNet lane (default 16; 64 for B >= 64)")
    ap.add_argument("--f16-steps", type=int, default=5, help="timed runs of the 16-bit sub-record")
    ap.add_argument("--f32-steps", type=int, default=2, help="timed runs of the fp32 sub-record")
    ap.add_argument("--workload", default="unet", choices=["unet", "diffwave", "wavegrad"])
    ap.add_argument("--num-samples", type=int, default=None,
                    help="UNet chunk length (config #5: 32832 = 512 frames); default config_unet.json's 16448")
    import sys as _sys
    args = ap.parse_args()
    args.batch_set = any(a.startswith("--batch") for a in _sys.argv[1:])
    args.timesteps_set = any(a.startswith("--timesteps") for a in _sys.argv[1:])
    if args.workload != "unet":
        return main_spec(args)

    import numpy as np
    import torch
    import torch.distributed as dist
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.network as module_network
    import model.model as module_arch
    from sddm_hip.synth import noisy_speech

    world, rank, dev = init_ranks()

    cfg = read_json(os.path.join(PKG, "configs", "config_unet_bench.json"))
    cfg["diffusion"]["args"]["n_timestep"] = args.timesteps
    if args.num_samples:
        cfg["num_samples"] = args.num_samples
    config = ConfigParser(cfg)
    N = config["num_samples"]
    T = args.timesteps
    B = args.batch
    torch.manual_seed(0)                                            # random-init weights
    diffusion = config.init_obj("diffusion", module_diffusion, device=dev)
    network = config.init_obj("network", module_network, num_samples=N)
    model = config.init_obj("arch", module_arch, diffusion, network).to(dev).eval()
    model.compute_dtype = DTYPE_NAMES[args.dtype]
    model.lane_rows = args.lane_rows or (64 if B >= 64 else None)  # 64-row lanes for large per-GPU batches

    cond_all = torch.from_numpy(noisy_speech(B * world, N, seed=1234)).to(dev)   # VoiceBank-DEMAND-shaped chunks
    result = {}

    def step():
        # the product multi-GPU path (model.model.sharded_infer): rank r samples rows
        # [rB, (r+1)B) with row_offset rB, then ONE RCCL all-gather of the outputs
        result["out"] = module_arch.sharded_infer(model, cond_all, seed=7)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() != "gloo" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if not torch.isfinite(result["out"]).all():
        raise RuntimeError("non-finite samples")

    roofline = None
    log(f"timed region: {elapsed:.2f} s")
    if rank == 0 and not args.no_profile:
        log("profiling one sampling run (HIP events around every launch)")
        roofline = unet_roofline(model, cond_all[:B].contiguous(), N, B, T, args.dtype, 1e3 * elapsed / args.steps)

    # same-run precision sub-records (N=1 only, after the timed region): the fp32 parity path and the
    # fp16 twin of the headline, each timed on the same workload, with the RMS drift of every
    # 16-bit output from the fp32 output of the same seed (north_star's bar: 1e-3)
    variants = None
    if (world == 1 and rank == 0 and not args.no_variants and args.dtype != "f32" and B <= 16
            and not args.num_samples):                             # the headline workload only
        main_out, main_dtype = result["out"], model.compute_dtype
        variants = {}
        v32 = unet_variant(model, step, result, "f32", args.f32_steps, 1, N, B, T, cond_all, args.no_profile)
        out32 = v32.pop("out")
        for dt in [d for d in ("f16", "bf16") if d != args.dtype]:
            v = unet_variant(model, step, result, dt, args.f16_steps, 1, N, B, T, cond_all, args.no_profile)
            v["drift_vs_f32_rms"] = rms(v.pop("out"), out32)
            variants[dt] = v
        variants["f32"] = v32
        drift_main = rms(main_out, out32)
        model.compute_dtype = main_dtype

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:   # CPU baseline: rank 0 at N=1 only
        log("CPU baseline")
        v, dt, threads, dt8 = cpu_baseline(B, args.cpu_steps, N, T)
        cpu_model, ncpu, naff = cpu_info()
        cpu = {"value": round(v, 6), "unit": "audio_s/s", "cores": threads, "kind": "port",
               "cpu_model": cpu_model, "cpu_count": ncpu, "cpu_affinity": naff, "cpu_quota_cores": cpu_quota(),
               "sample": f"PyTorch-CPU restatement of UNetModified2 (oracle/unet_torch.py, pinned to the "
                         f"reference goldens), {args.cpu_steps} reverse steps at B={B}x{N} ({dt:.2f} s/step, "
                         f"torch.set_num_threads({threads})), extrapolated x{T}/{args.cpu_steps}",
               "note": "the GPU box shares its host: os.cpu_count() shows the whole machine, the job runs under "
                       "a CPU quota (cpu_quota_cores) beside other jobs, so this understates an idle host (the "
                       "survey timed the reference itself at 0.654 s/step on 8 idle Xeon threads)"}
        if dt8 is not None:
            cpu["threads_8"] = {"s_per_step": round(dt8, 3), "value": round(B * N / 16000.0 / (dt8 * T), 6)}

    if rank == 0:
        audio_s = args.steps * B * world * N / 16000.0
        line = {"metric": f"denoised audio sec/sec, {T}-step UNetModified2 @16kHz",
                "value": round(audio_s / elapsed, 4), "unit": "audio_s/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                "data": "synthetic (harmonic speech + gaussian noise, 16 kHz), random-init weights",
                "config": {"workload": f"UNetModified2 config_unet.json, linear 1e-6..1e-3, T={T}, "
                                       f"{B}x{N}-sample chunks per GPU, condition_in",
                           "model": "UNetModified2", "global_batch": B * world, "seq_len": N,
                           "timesteps": T, "parallelism": f"dp{world}", "lane_rows": model.lane_rows or 16},
                "roofline": roofline, "cpu_baseline": cpu}
        if variants is not None:
            line["drift_vs_f32_rms"] = drift_main
            line["variants"] = variants
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
