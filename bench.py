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

Rank 0 prints one JSON line.  `roofline` is measured with HIP events around every conv3x3
launch of one extra (untimed) sampling run; `cpu_baseline` times the numpy oracle on a bounded
sample of the same workload on this host's cores.
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


def cpu_baseline(B_cpu, k_steps, N, T, threads):
    """numpy oracle (tests-only restatement of the reference) timed on the host cores."""
    sys.path.insert(0, REPO)
    import numpy as np
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    from oracle import philox, sampler, schedule, unet
    from sddm_hip.synth import noisy_speech
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from _weights import make_params, unet_shapes
    arch = unet.architecture(N, inner_channel=32, channel_mults=(1, 2, 3, 4, 5), res_blocks=1)
    P = make_params(unet_shapes(arch), 0)
    tab = schedule.make_tables("linear", T, 1e-6, 1e-3)
    cond = noisy_speech(B_cpu, N, seed=1234)
    x = sampler.get_x_T(tab, cond, philox.normal(7, 0, cond.shape))
    unet.forward(P, arch, cond, x, np.full(B_cpu, tab["sqrt_alpha_bar"][T], np.float32))  # warm BLAS
    t0 = time.perf_counter()
    for i in range(k_steps):
        t = T - i
        eps = unet.forward(P, arch, cond, x, np.full(B_cpu, tab["sqrt_alpha_bar"][t], np.float32))
        x = sampler.transition("condition_in", tab, x, t, eps, cond, philox.normal(7, t, x.shape))
    dt = (time.perf_counter() - t0) / k_steps
    return B_cpu * N / 16000.0 / (dt * T), dt


# spectrogram-conditioned workloads (BASELINE.json configs #3 and #4): config, frames, clips per GPU,
# step-variant GFLOP per clip and step
SPEC_WORKLOADS = {
    "diffwave": dict(config="config_diffwave_bench.json", frames=63, batch=64, bins=513, gflop=31.85,
                     label="DiffWave config_diffwave.json, linear 1e-4..0.02, T=200, time_step conditioning"),
    "wavegrad": dict(config="config_wavegrad_bench.json", frames=54, batch=64, bins=128, gflop=47.38,
                     label="WaveGrad, linear 1e-4..0.05, T=50 (SURVEY §8d fast schedule), sqrt_alpha_bar"),
}


def cpu_baseline_spec(workload, model, spec_np, T, threads):
    """numpy oracle forward of one clip for one step, extrapolated x T (tests-only restatement)."""
    sys.path.insert(0, REPO)
    import numpy as np
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
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
    diffusion = config.init_obj("diffusion", module_diffusion, device=dev)
    network = config.init_obj("network", module_network, num_samples=N, num_timesteps=T, freq_bins=W["bins"])
    if args.workload == "diffwave":                                 # output_projection is zero-init
        with torch.no_grad():
            network.output_projection.weight.uniform_(-0.1, 0.1)
    extra = {} if "hop_samples" in cfg["arch"]["args"] else {"hop_samples": hop}
    model = config.init_obj("arch", module_arch, diffusion, network, **extra).to(dev).eval()
    model.compute_dtype = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}[args.dtype]
    rng = np.random.default_rng(1234)
    spec_all = rng.uniform(0, 1, (B * world, W["bins"], F)).astype(np.float32)   # U[0,1]
    spec = torch.from_numpy(spec_all[rank * B:(rank + 1) * B]).to(dev)
    gathered = torch.empty((B * world, 1, N), dtype=torch.float32, device=dev)

    def step():
        out = model.infer(spec, seed=7, row_offset=rank * B)
        if world > 1:
            dist.all_gather_into_tensor(gathered, out)
        else:
            gathered.copy_(out)

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
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if not torch.isfinite(gathered).all():
        raise RuntimeError("non-finite samples")
    if rank == 0:
        tfs = args.steps * T * B * W["gflop"] / elapsed / 1e3      # whole-job MFMA rate per GPU
        cpu = None
        if not args.no_cpu_baseline:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
            v, dt, reps = cpu_baseline_spec(args.workload, model, spec_all, T, threads)
            cpu = {"value": round(v, 6), "unit": "audio_s/s", "cores": threads, "kind": "port",
                   "sample": f"numpy oracle, {reps} network evaluations of 1 clip ({dt:.2f} s each), "
                             f"extrapolated x{T} steps"}
        audio_s = args.steps * B * world * N / 16000.0
        line = {"metric": f"denoised audio sec/sec, {T}-step {network.__class__.__name__} @16kHz",
                "value": round(audio_s / elapsed, 4), "unit": "audio_s/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                "data": "synthetic spectrograms U[0,1], random-init weights",
                "config": {"workload": f"{W['label']}, {B}x{N}-sample clips per GPU",
                           "model": network.__class__.__name__, "global_batch": B * world, "seq_len": N,
                           "timesteps": T, "parallelism": f"dp{world}"},
                "roofline": {"bound": "mfma", "achieved": round(tfs, 2),
                             "peak": MFMA_PEAK_TFLOPS[args.dtype], "unit": "TFLOP/s",
                             "frac": round(tfs / MFMA_PEAK_TFLOPS[args.dtype], 4), "traffic": None,
                             "kernel": "whole sampling run (step-variant algorithmic FLOPs / wall)"},
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
    ap.add_argument("--cpu-batch", type=int, default=2)
    ap.add_argument("--cpu-steps", type=int, default=25, help="oracle reverse steps (~10 s of host work)")
    ap.add_argument("--no-profile", action="store_true")
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

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

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
    model.compute_dtype = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}[args.dtype]

    cond_all = noisy_speech(B * world, N, seed=1234)                 # VoiceBank-DEMAND-shaped chunks
    cond = torch.from_numpy(cond_all[rank * B:(rank + 1) * B]).to(dev)
    gathered = torch.empty((B * world, 1, N), dtype=torch.float32, device=dev)

    def step():
        out = model.infer(cond, seed=7, row_offset=rank * B)
        if world > 1:
            dist.all_gather_into_tensor(gathered, out)              # one RCCL all-gather
        else:
            gathered.copy_(out)

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
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if not torch.isfinite(gathered).all():
        raise RuntimeError("non-finite samples")

    roofline = None
    prof = {}
    if rank == 0 and not args.no_profile:
        ctx = model._context(dev)
        ctx.profile(True)
        model.infer(cond, seed=7, row_offset=0)
        torch.cuda.synchronize()
        for cls in ("conv3x3", "gn_finalize", "final", "conv_in"):
            prof[cls] = ctx.profile_read(cls)
        ctx.profile(False)
        p = prof["conv3x3"]
        if p["launches"]:
            gbs = p["bytes_per_launch"] / (p["avg_ms"] * 1e-3) / 1e9
            tfs = p["flops_per_launch"] / (p["avg_ms"] * 1e-3) / 1e12
            # measured HBM bytes per conv launch: the committed PMC summary of the same workload
            # (tools/gpu_traffic.sh + tools/traffic.py; counters cannot be read from inside this run)
            traffic, tsrc = None, None
            tf = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "hbm_traffic.json")
            if os.path.exists(tf) and (N, B, args.dtype, T) == (16448, 16, "bf16", 1000):   # the PMC workload
                with open(tf) as fh:
                    traffic = round(json.load(fh)["bytes_per_launch"])
                tsrc = "profiles/hbm_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, same workload)"
            roofline = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                        "kernel": "conv3x3_kernel (all UNet 3x3 conv launches)",
                        "avg_launch_ms": round(p["avg_ms"], 5), "launches_timed": p["launches"],
                        "alg_bytes_per_launch": round(p["bytes_per_launch"]),
                        "mfma_tflops": round(tfs, 2), "mfma_frac": round(tfs / MFMA_PEAK_TFLOPS[args.dtype], 4)}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        v, dt = cpu_baseline(args.cpu_batch, args.cpu_steps, N, T, threads)
        cpu = {"value": round(v, 6), "unit": "audio_s/s", "cores": threads, "kind": "port",
               "sample": f"numpy oracle, {args.cpu_steps} reverse steps at B={args.cpu_batch}x{N} "
                         f"({dt:.2f} s/step), extrapolated x{T}/step"}

    if rank == 0:
        audio_s = args.steps * B * world * N / 16000.0
        line = {"metric": "denoised audio sec/sec, 1000-step UNetModified2 @16kHz",
                "value": round(audio_s / elapsed, 4), "unit": "audio_s/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
                "data": "synthetic (harmonic speech + gaussian noise, 16 kHz), random-init weights",
                "config": {"workload": f"UNetModified2 config_unet.json, linear 1e-6..1e-3, T={T}, "
                                       f"{B}x{N}-sample chunks per GPU, condition_in",
                           "model": "UNetModified2", "global_batch": B * world, "seq_len": N,
                           "timesteps": T, "parallelism": f"dp{world}"},
                "roofline": roofline, "cpu_baseline": cpu}
        if prof:
            line["kernel_classes_ms"] = {k: round(v["avg_ms"], 5) for k, v in prof.items()}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
