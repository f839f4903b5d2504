"""Measure the narrow-level conv tile per UNet layer and write the tuning table the facade hands to
the library (sddm_set_conv_tuning).

    python tools/tune_deep.py [--batch 16] [--dtype bf16] [--out <pkg>/configs/conv_tuning.json]
    python tools/tune_deep.py --from-dir gpurun_out      # reuse deep_<cfg>.json files

Each candidate (pixels per block, waves) is forced on every layer with SDDM_DEEP_CFG in a child
process running tools/profile_ops.py (HIP events around every launch of a short sampling run); a
layer takes the candidate that beats the heuristic's own choice by >= 1 us.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CANDS = ["default", "128:8", "128:4", "64:8", "64:4", "32:8", "32:4"]
DT = {"bf16": "bfloat16", "f16": "float16", "f32": "float32"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--num-samples", type=int, default=16448)
    ap.add_argument("--from-dir", default=None)
    ap.add_argument("--out", default=os.path.join(REPO, "speech-denoising-diffusion-model-2_amd", "configs",
                                                  "conv_tuning.json"))
    a = ap.parse_args()
    d = a.from_dir or os.path.join(REPO, "gpurun_out")
    if not a.from_dir:
        for c in CANDS:
            env = dict(os.environ)
            if c != "default":
                env["SDDM_DEEP_CFG"] = c
            subprocess.run([sys.executable, os.path.join(REPO, "tools", "profile_ops.py"), "--batch", str(a.batch),
                            "--dtype", a.dtype, "--json", os.path.join(d, f"deep_{c}.json")], env=env, check=True)
    D = {c: {o["name"]: o["avg_ms"] * 1e3 for o in json.load(open(os.path.join(d, f"deep_{c}.json")))} for c in CANDS}
    deep = {}
    for name, base in D["default"].items():
        if "[strip]" in name or name in ("downs.0", "final_conv"):
            continue
        best = min(CANDS[1:], key=lambda c: D[c].get(name, 1e9))
        if D[best].get(name, 1e9) <= base - 1.0:
            deep[name] = [int(x) for x in best.split(":")]
            print(f"{name:20s} {base:6.1f} -> {D[best][name]:6.1f} us ({best})")
    table = {"lane_batch": a.batch, "dtype": DT[a.dtype], "num_samples": a.num_samples, "deep": deep}
    with open(a.out, "w") as f:
        json.dump(table, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
