"""Per-launch HBM traffic of the 3x3 conv kernels from tools/gpu_traffic.sh counter dumps.

FETCH_SIZE is doubled (gfx950 tallies the 128-B requests of 16-B/lane streaming reads at 64 B,
MI355X_MICROARCH.md 'HBM'); WRITE_SIZE is taken as is.  Both are reported by rocprofv3 in KB.
Writes profiles/<name>.json with the per-class averages and the per-kernel rows."""
import csv, glob, json, os, re, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "hbm_traffic.json")


def rows(counter):
    f = glob.glob(os.path.join(REPO, "gpurun_out", f"traffic_{counter}", "**", "*counter_collection.csv"), recursive=True)
    if not f:
        sys.exit(f"no counter dump for {counter}")
    r = {}
    for x in csv.DictReader(open(f[0])):
        key = int(x["Dispatch_Id"])
        r.setdefault(key, {"name": x["Kernel_Name"], "v": 0.0})
        r[key]["v"] += float(x["Counter_Value"])
    return [r[k] for k in sorted(r)]


fe, wr = rows("FETCH_SIZE"), rows("WRITE_SIZE")
if len(fe) != len(wr):
    sys.exit("dispatch counts differ between the passes")
conv = [(f["name"], 2 * f["v"] * 1024, w["v"] * 1024) for f, w in zip(fe, wr) if re.search(r"conv_(strip|deep)", f["name"])]
tot = [a + b for _, a, b in conv]
res = {"what": "HBM bytes per 3x3 conv launch (conv_strip + conv_deep), one sampling step, B=16x16448, bf16",
       "counters": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) and --pmc WRITE_SIZE, separate passes",
       "launches": len(conv), "read_bytes_per_launch": statistics.mean(a for _, a, _ in conv),
       "write_bytes_per_launch": statistics.mean(b for _, _, b in conv),
       "bytes_per_launch": statistics.mean(tot),
       "per_launch": [{"kernel": n[:80], "read": round(a), "write": round(b)} for n, a, b in conv]}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "per_launch"}))
