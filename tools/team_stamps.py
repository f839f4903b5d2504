"""Per-op timeline of the deep-level team kernel from its per-item timestamps (SDDM_TEAM_STAMPS=1).

    python tools/team_stamps.py [--batch 16] [--dtype bf16]

Runs one bench-geometry network forward, reads the stamps ({op | b << 16, ticket, after wait,
publish} per item, s_memrealtime 100 MHz) and prints per op: items, first ticket / last publish
relative to the launch's first ticket, mean wait and mean item time (us).
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SDDM_TEAM_STAMPS"] = "1"
sys.path.insert(0, os.path.join(REPO, "speech-denoising-diffusion-model-2_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--N", type=int, default=16448)
    a = ap.parse_args()
    import numpy as np
    import torch
    import sddm_hip
    from _helpers import unet_config, unet_params
    from sddm_hip.synth import noisy_speech
    dt = {"bf16": "bfloat16", "f16": "float16"}[a.dtype]
    ctx = sddm_hip.Context(unet_config(a.N, ("linear", 1000, 1e-6, 1e-3)), 0, dt)
    for k, v in unet_params(a.N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    dev = torch.device("cuda", 0)
    cond = torch.from_numpy(noisy_speech(a.batch, a.N)).to(dev)
    x = torch.randn_like(cond)
    nl = torch.full((a.batch,), 0.5, device=dev)
    eps = torch.empty_like(cond)
    names = [o["name"] for o in ctx.profile_ops()] if False else None
    L = sddm_hip.lib()
    L.sddm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.sddm_debug_stamps.restype = ctypes.c_int
    for rep in range(3):
        ctx.network_forward(cond, x, nl, eps)
        torch.cuda.synchronize()
    buf = np.zeros((65536, 8), dtype=np.uint64)
    n = ctypes.c_int64()
    sddm_hip.check(L.sddm_debug_stamps(ctx._h, buf.ctypes.data, 65536, ctypes.byref(n)))
    st = buf[: n.value].reshape(-1, 8)
    st = st[st[:, 1] > 0]
    t0 = st[:, 1].min()
    ops = (st[:, 0] & 0xFFFF).astype(int)
    print(f"{len(st)} items, launch span {(st[:, 3].max() - t0) / 100:.1f} us")
    print(" op  items  first-ticket  last-publish  span   mean-wait  item: gnfin  staged kloop  stats  publish (us after the wait)")
    prev_end = 0.0
    for o in sorted(set(ops)):
        m = st[ops == o]
        first = (m[:, 1].min() - t0) / 100
        last = (m[:, 3].max() - t0) / 100
        wait = ((m[:, 2] - m[:, 1]) / 100).mean()
        item = ((m[:, 3] - m[:, 2]) / 100).mean()
        ph = [((m[:, k] - m[:, 2]) / 100).mean() for k in (4, 5, 6, 7, 3)]
        print(f"{o:3d} {len(m):6d} {first:12.1f} {last:13.1f} {last - prev_end:6.1f} {wait:10.2f}       "
              + "  ".join(f"{x:5.2f}" for x in ph))
        prev_end = last


if __name__ == "__main__":
    main()
