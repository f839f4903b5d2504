"""Per-kernel PMC summary of gpu_pmc2.sh passes: the last sampling step's dispatches in order."""
import csv, glob, sys
from collections import OrderedDict
disp = OrderedDict()
for f in sorted(glob.glob("gpurun_out/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        key = (f.split("/")[1], int(r["Dispatch_Id"]))
        d = disp.setdefault(key, {"name": r["Kernel_Name"], "grid": r["Grid_Size"], "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
# group per pass, keep sddm kernels of the last 44 conv-ish dispatches
passes = sorted({k[0] for k in disp})
for p in passes:
    rows = [v for k, v in disp.items() if k[0] == p and "sddm" in v["name"] and ("conv" in v["name"] or "final" in v["name"])]
    rows = rows[-44:]
    keys = [k for k in rows[0] if k not in ("name", "grid", "dur")]
    print(p, "kernel".ljust(28), "dur_us".rjust(7), "".join(k.replace("SQ_", "")[:14].rjust(15) for k in keys))
    for v in rows:
        nm = v["name"].replace("_ZN4sddm", "").replace("void sddm::", "")[:28]
        print(p, nm.ljust(28), f"{v['dur']:7.1f}", "".join(f"{v.get(k, 0):15.4g}" for k in keys))
