"""Summarize gpu_ablate.sh traces: median duration of the relaunched (ablated) layer launches."""
import csv, glob, os, re, statistics, sys
rows = {}
for d in sorted(glob.glob("gpurun_out/abl_*_*")):
    if not os.path.isdir(d):
        continue
    m = re.match(r"gpurun_out/abl_(.+)_(\d+)$", d)
    op, fl = m.group(1), int(m.group(2))
    f = glob.glob(d + "/*kernel_trace.csv")
    if not f:
        continue
    k = list(csv.DictReader(open(f[0])))
    k.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = []
    i = 0
    while i < len(k):
        j = i
        while j + 1 < len(k) and k[j + 1]["Kernel_Name"] == k[i]["Kernel_Name"]:
            j += 1
        if j - i + 1 >= 4:
            durs += [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in k[i + 1:j + 1]]
        i = j + 1
    rows.setdefault(op, {})[fl] = statistics.median(durs) if durs else float("nan")
names = {0: "full", 1: "-stats", 2: "-GN", 4: "-res/temb", 8: "-Kloop", 15: "-all"}
fls = sorted({f for v in rows.values() for f in v})
print("layer".ljust(18) + "".join(names.get(f, str(f)).rjust(11) for f in fls))
for op, v in rows.items():
    print(op.ljust(18) + "".join(f"{v.get(f, float('nan')):11.2f}" for f in fls))
