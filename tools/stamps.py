"""Per-block phase timestamps of selected conv launches (profiling build, SDDM_STAMPS).

    SDDM_BUILD_VARIANT=stamps python speech-denoising-diffusion-model-2_amd/sddm_hip/build.py
    python tools/stamps.py [--batch 16] [--dtype bf16] op1 op2 ...

Stamps (conv_common.h SDDM_STAMP): s_memrealtime (100 MHz) at block start (0), end (7) and
the phase boundaries (1..6) (deep kernel: 1 staging loads issued, 2 GroupNorm
finalized, 3 LDS image written, 4 K loop done, 5 epilogue stored, 6 stats written; strip kernel:
3 initial rows staged, 4 row loop done, 6 stats written).
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("SDDM_LIB", os.path.join(REPO, "tools", "_stamps", "libsddm_hip.so"))
sys.path.insert(0, os.path.join(REPO, "speech-denoising-diffusion-model-2_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--N", type=int, default=16448)
    ap.add_argument("ops", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    import sddm_hip
    from _helpers import unet_config, unet_params
    from sddm_hip.synth import noisy_speech
    dt = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}[a.dtype]
    dev = torch.device("cuda", 0)
    L = sddm_hip.lib()
    L.sddm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.sddm_debug_stamps.restype = ctypes.c_int
    params = unet_params(a.N)
    cond = torch.from_numpy(noisy_speech(a.batch, a.N, seed=3)).to(dev)
    x = torch.from_numpy(noisy_speech(a.batch, a.N, seed=4)).to(dev)
    nl = torch.full((a.batch,), 0.5, device=dev)
    eps = torch.empty_like(cond)
    for op in a.ops:
        os.environ["SDDM_STAMPS"] = op
        ctx = sddm_hip.Context(unet_config(a.N), 0, dt)
        tf = os.path.join(REPO, "speech-denoising-diffusion-model-2_amd", "configs", "conv_tuning.json")
        if os.path.exists(tf) and not os.environ.get("SDDM_NO_TUNING"):    # the measured per-layer kernels
            with open(tf) as f:
                ctx.set_conv_tuning(f.read())
        for k, v in params.items():
            ctx.load_param("noise_estimate_model." + k, v)
        for _ in range(3):
            ctx.network_forward(cond, x, nl, eps)
        torch.cuda.synchronize()
        buf = np.zeros((65536, 8), dtype=np.uint64)
        n = ctypes.c_int64()
        sddm_hip.check(L.sddm_debug_stamps(ctx._h, buf.ctypes.data, 65536, ctypes.byref(n)))
        st = buf[:n.value].astype(np.float64)
        if n.value == 0:
            print(op, "no stamps")
            continue
        t0, t7 = st[:, 0], st[:, 7]
        span = (t7.max() - t0.min()) * 10e-3
        dur = (t7 - t0) * 10e-3
        start = (t0 - t0.min()) * 10e-3
        nz = [0] + [k for k in range(1, 7) if st[:, k].any()] + [7]
        ph = [f"{k0}->{k1}: {np.mean(st[:, k1] - st[:, k0]) * 10e-3:6.2f}" for k0, k1 in zip(nz[:-1], nz[1:])]
        ev = sorted([(x, 1) for x in t0] + [(x, -1) for x in t7], key=lambda e: (e[0], e[1]))
        cur = conc = 0
        for _, d in ev:
            cur += d
            conc = max(conc, cur)
        print(f"{op}: {n.value} blocks, span {span:.1f} us, block dur mean {dur.mean():.2f} max {dur.max():.2f} us, "
              f"start spread max {start.max():.2f} us (p50 {np.median(start):.2f}), max concurrent blocks {conc}")
        print("   us " + "  ".join(ph))
        ctx.close()


if __name__ == "__main__":
    main()
