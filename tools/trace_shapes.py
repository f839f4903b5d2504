"""Per (kernel, grid) time table from a rocprofv3 kernel trace CSV: trace_shapes.py <csv> [name filter]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    if filt not in r["Kernel_Name"]:
        continue
    k = (r["Kernel_Name"][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    tot += v[1]
    print("%4d %9.1f us  avg %7.1f  %s" % (v[0], v[1], v[1] / v[0], k))
print("total %.1f us" % tot)
