"""Summarise rocprofv3 --pmc CSVs per (kernel, grid) : python tools/pmc_table.py gpurun_out/pmc1 gpurun_out/pmc2"""
import collections
import csv
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        name = r["Kernel_Name"]
        m = re.search(r"sddm(?:17|16|14|12)?([a-z_]+)", name)
        short = (m.group(1) if m else name)[:18]
        tmpl = re.findall(r"Li(\d+)E", name)
        key = (short + ("<" + ",".join(tmpl) + ">" if tmpl else ""), int(r["Grid_Size"]))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[key]["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        meta[key] = (r["LDS_Block_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"])
cols = ["dur_us", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT"]
cols = [c for c in cols if any(c in v for v in agg.values())]
print(f"{'kernel':34s} {'grid':>8s} {'lds':>6s} {'vgpr':>5s} " + " ".join(f"{c.replace('SQ_', '')[:12]:>12s}" for c in cols))
for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]["dur_us"]) / max(len(kv[1]["dur_us"]), 1)):
    if "sddm" not in key[0] and not key[0].startswith(("conv", "final", "embed")):
        pass
    vals = []
    for c in cols:
        x = v.get(c, [])
        vals.append(sum(x) / len(x) if x else float("nan"))
    print(f"{key[0]:34s} {key[1]:8d} {meta[key][0]:>6s} {meta[key][1]:>5s} " + " ".join(f"{x:12.4g}" for x in vals))
