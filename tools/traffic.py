"""Per-launch HBM traffic of every UNet kernel from tools/gpu_traffic.sh counter dumps.

FETCH_SIZE is doubled (gfx950 tallies the 128-B requests of 16-B/lane streaming reads at 64 B,
MI355X_MICROARCH.md 'HBM'); WRITE_SIZE is taken as is; rocprofv3 reports both in KB.  The last
step's dispatches of the profiled run are matched, in order, to the op list tools/profile_ops.py
wrote in the same pass; the summary is keyed by workload and kernel-source hash so that bench.py
reports `roofline.traffic` only for the kernels it measured."""
import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "r04_hbm_traffic.json")
# workload key (bench.py matches it): N, per-GPU batch, dtype; defaults = the headline config #2
N_ = int(sys.argv[2]) if len(sys.argv) > 2 else 16448
B_ = int(sys.argv[3]) if len(sys.argv) > 3 else 16
DT_ = sys.argv[4] if len(sys.argv) > 4 else "bf16"
UNET = re.compile(r"conv_in_kernel|conv_strip_kernel|conv_tile_kernel|conv_deep_kernel|final_kernel")


def dispatches(counter):
    f = glob.glob(os.path.join(REPO, "gpurun_out", f"traffic_{counter}", "**", "*counter_collection.csv"), recursive=True)
    if not f:
        sys.exit(f"no counter dump for {counter}")
    r = {}
    for x in csv.DictReader(open(f[0])):
        if not UNET.search(x["Kernel_Name"]):
            continue
        key = int(x["Dispatch_Id"])
        r.setdefault(key, {"name": x["Kernel_Name"], "kb": 0.0})
        r[key]["kb"] += float(x["Counter_Value"])
    return [r[k] for k in sorted(r)]


ops = json.load(open(os.path.join(REPO, "gpurun_out", "traffic_ops_FETCH_SIZE.json")))
fe, wr = dispatches("FETCH_SIZE")[-len(ops):], dispatches("WRITE_SIZE")[-len(ops):]
if len(fe) != len(ops) or len(wr) != len(ops):
    sys.exit("dispatch counts do not cover one step")
per_op, kern = [], {}
for o, f, w in zip(ops, fe, wr):
    rd, wb = 2 * f["kb"] * 1024, w["kb"] * 1024
    per_op.append({"op": o["name"], "kernel": o["kernel"], "alg_bytes": round(o["bytes"]), "read": round(rd),
                   "write": round(wb), "ratio": round((rd + wb) / o["bytes"], 3) if o["bytes"] else None})
    k = kern.setdefault(o["kernel"], {"n": 0, "bytes": 0.0, "alg": 0.0})
    k["n"] += 1
    k["bytes"] += rd + wb
    k["alg"] += o["bytes"]
from bench import kernel_src_hash  # noqa: E402
res = {"N": N_, "B": B_, "dtype": DT_, "src": kernel_src_hash(),
       "what": f"HBM bytes per launch of every UNet kernel, one reverse step, B={B_} x {N_}, {DT_}",
       "counters": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and --pmc WRITE_SIZE, separate passes",
       "step_bytes": round(sum(p["read"] + p["write"] for p in per_op)),
       "step_alg_bytes": round(sum(p["alg_bytes"] for p in per_op)),
       "kernels": {k: {"launches": v["n"], "bytes_per_launch": round(v["bytes"] / v["n"]),
                       "alg_bytes_per_launch": round(v["alg"] / v["n"]), "ratio": round(v["bytes"] / v["alg"], 3)}
                   for k, v in kern.items()},
       "per_op": per_op}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("step_bytes", "step_alg_bytes", "src")}),
      "ratio", round(res["step_bytes"] / res["step_alg_bytes"], 3))
