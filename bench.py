#!/usr/bin/env python
"""Bench: denoised-audio seconds per second of 1000-step reverse diffusion with UNetModified2
(BASELINE.json metric; config_unet.json network, linear 1e-6..1e-3 schedule at T=1000).

One bench *step* = one full SDDM.infer sampling run (x_T -> x_0, T UNet evaluations + T
transitions) of a per-GPU batch of B synthetic 16 kHz chunks (16448 samples = 256 frames), entered
through the drop-in facade (model.model.SDDM.infer -> libsddm_hip).  With N GPUs every rank samples
its own B rows (row_offset = rank * B, so results equal a single-GPU run of all rows) and the
outputs are all-gathered over RCCL at the end of the step (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--timesteps T] [--dtype bf16]

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
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

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
            if os.path.exists(tf):
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
                                       f"{B}x16448-sample chunks per GPU, condition_in",
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
