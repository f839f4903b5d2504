"""Merge per-layer timings of a conv kernel sweep (tools/gpu_tile_sweep.sh) and pick the fastest
kernel per layer: prints the table and the step total with the per-layer best."""
import glob
import json
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep"
runs = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    runs[os.path.basename(f)[:-5]] = {re.sub(r"\[.*\]", "", o["name"]): (o["avg_ms"] * 1e3, o["name"]) for o in json.load(open(f))}
layers = list(runs["deep"].keys())
tot_best, tot_deep, tot_auto = 0.0, 0.0, 0.0
pick = {}
for L in layers:
    cands = {k: v[L] for k, v in runs.items() if L in v}
    best = min(cands.items(), key=lambda kv: kv[1][0])
    tot_best += best[1][0]
    tot_deep += cands["deep"][0]
    tot_auto += cands["auto"][0]
    pick[L] = best[1][1]
    row = "  ".join(f"{k}:{v[0]:6.1f}" for k, v in sorted(cands.items()) if k in ("deep", "auto"))
    print(f"{L:16s} best {best[1][0]:6.1f} {best[1][1]:26s} {row}")
print(f"step total: deep {tot_deep:.1f}  auto {tot_auto:.1f}  best-per-layer {tot_best:.1f} us")
if len(sys.argv) > 2:       # write the per-layer table for sddm_set_conv_tuning
    kern = {}
    for L, name in pick.items():
        m = re.search(r"\[(strip|tile(\d+)|deep(\d+)_(\d+)_(\d+))\]", name)
        if m is None:
            kern[L] = "deep"
        elif m.group(1) == "strip":
            kern[L] = "strip"
        elif m.group(2) is not None:
            kern[L] = "tile:" + m.group(2)
        else:
            kern[L] = "deep:%s:%s:%s" % (m.group(3), m.group(4), m.group(5))
    if "downs.0" in kern:
        del kern["downs.0"]
    kern.pop("final_conv", None)
    lane_batch = int(os.environ.get("SWEEP_LANE_BATCH", "16"))
    out = {"lane_batch": lane_batch, "dtype": os.environ.get("SWEEP_DTYPE", "bfloat16"),
           "num_samples": int(os.environ.get("SWEEP_NUM_SAMPLES", "16448")),
           "source": "tools/gpu_tile_sweep.sh + tools/sweep_merge.py (fastest measured kernel per layer)",
           "kernel": kern}
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print("wrote", sys.argv[2])
