"""Per-op timestamps inside the fused deep-level chain (conv_chain.hip), normal build.

    SDDM_CHAIN_STAMPS=1 python tools/chain_stamps.py [--batch 16] [--dtype bf16]

Per image: s_memrealtime (100 MHz) at each op's start and at the end of its K loop, and at the
kernel's end; printed as the median over images of the K-loop time and the epilogue time per op.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speech-denoising-diffusion-model-2_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--N", type=int, default=16448)
    a = ap.parse_args()
    os.environ["SDDM_CHAIN_STAMPS"] = "1"
    os.environ.setdefault("SDDM_CHAIN", "1")
    import numpy as np
    import torch
    import sddm_hip
    from _helpers import unet_config, unet_params
    from sddm_hip.synth import noisy_speech
    dt = {"bf16": "bfloat16", "f16": "float16"}[a.dtype]
    dev = torch.device("cuda", 0)
    L = sddm_hip.lib()
    L.sddm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.sddm_debug_stamps.restype = ctypes.c_int
    ctx = sddm_hip.Context(unet_config(a.N), 0, dt)
    for k, v in unet_params(a.N).items():
        ctx.load_param("noise_estimate_model." + k, v)
    cond = torch.from_numpy(noisy_speech(a.batch, a.N, seed=3)).to(dev)
    x = torch.from_numpy(noisy_speech(a.batch, a.N, seed=4)).to(dev)
    nl = torch.full((a.batch,), 0.5, device=dev)
    eps = torch.empty_like(cond)
    for _ in range(3):
        ctx.network_forward(cond, x, nl, eps)
    torch.cuda.synchronize()
    names = [o["name"] for o in ctx.profile_ops()]
    print("ops:", [n for n in names if n.startswith("chain")])
    buf = np.zeros((65536, 8), dtype=np.uint64)
    n = ctypes.c_int64()
    sddm_hip.check(L.sddm_debug_stamps(ctx._h, buf.ctypes.data, 65536, ctypes.byref(n)))
    st = buf[:n.value].reshape(a.batch, 64).astype(np.float64) * 0.01   # us
    nops = int(os.environ.get("CHAIN_NOPS", "14"))
    total = np.median(st[:, 63] - st[:, 0])
    print(f"chain total (median over images) {total:.1f} us")
    print("  op: prologue (GN + first staging) | K loop | epilogue | to next op")
    for i in range(nops):
        s0, s1, s2, s3 = (st[:, 4 * i + k] for k in range(4))
        nxt = st[:, 4 * i + 4] if i + 1 < nops else st[:, 63]
        if s1[0] == 0:   # reload op
            print(f"  op {i:2d}: reload {np.median(nxt - s0):6.2f} us")
            continue
        print(f"  op {i:2d}: {np.median(s1 - s0):6.2f} | {np.median(s2 - s1):7.2f} | {np.median(s3 - s2):6.2f} | {np.median(nxt - s3):5.2f}")


if __name__ == "__main__":
    main()
