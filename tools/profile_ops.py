"""Per-layer timing of one sampling run (HIP events around every launch).

    python tools/profile_ops.py [--batch 16] [--timesteps 20] [--dtype bf16] [--num-samples N] [--lane-rows R]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speech-denoising-diffusion-model-2_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--timesteps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--json", default=None)
    ap.add_argument("--num-samples", type=int, default=None, help="chunk length (default: the bench config's)")
    ap.add_argument("--lane-rows", type=int, default=None, help="rows per lane (bench.py: 64 for batches of 64+)")
    a = ap.parse_args()
    import torch
    from parse_config import ConfigParser, read_json
    import model.diffusion as module_diffusion
    import model.network as module_network
    import model.model as module_arch
    from sddm_hip.synth import noisy_speech
    dev = torch.device("cuda", 0)
    cfg = read_json(os.path.join(REPO, "speech-denoising-diffusion-model-2_amd", "configs", "config_unet_bench.json"))
    cfg["diffusion"]["args"]["n_timestep"] = a.timesteps
    if a.num_samples:
        cfg["num_samples"] = a.num_samples
    config = ConfigParser(cfg)
    N = config["num_samples"]
    torch.manual_seed(0)
    d = config.init_obj("diffusion", module_diffusion, device=dev)
    n = config.init_obj("network", module_network, num_samples=N)
    m = config.init_obj("arch", module_arch, d, n).to(dev)
    m.compute_dtype = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}[a.dtype]
    m.lane_rows = a.lane_rows
    cond = torch.from_numpy(noisy_speech(a.batch, N)).to(dev)
    m.infer(cond, seed=1)
    ctx = m._context(dev)
    ctx.profile(True)
    m.infer(cond, seed=1)
    torch.cuda.synchronize()
    ops = ctx.profile_ops()
    ctx.profile(False)
    tot = sum(o["avg_ms"] for o in ops)
    print(f"per-step total of launch durations: {tot * 1e3:.1f} us over {len(ops)} launches (B={a.batch}, {a.dtype})")
    for o in sorted(ops, key=lambda o: -o["avg_ms"]):
        t = o["avg_ms"] * 1e-3
        gbs = o["bytes"] / t / 1e9 if t else 0
        tfs = o["flops"] / t / 1e12 if t else 0
        print(f"{o['avg_ms'] * 1e3:8.2f} us  {100 * o['avg_ms'] / tot:5.1f}%  {gbs:7.1f} GB/s {tfs:7.2f} TF/s  {o['name']}")
    if a.json:
        json.dump(ops, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
