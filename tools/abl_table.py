"""Summarize gpu_ablate.sh traces: the relaunched (ablated) copies of one layer.

Launch order of one network pass = UNetModified2 layer order (conv_in = downs.0, ResnetBlocks
as .block1/.block2, final_conv last); SDDM_REPEAT_OP relaunches layer i right after itself, so
the ablated copies are conv launches i+1 .. i+N of the first pass."""
import csv, glob, os, re, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "speech-denoising-diffusion-model-2_amd")]
from _helpers import unet_arch
arch = unet_arch(16448)
order = []
for kind, name, *_ in arch["downs"] + arch["mid"] + arch["ups"]:
    order += [name + ".block1", name + ".block2"] if kind == "res" else [name]
order.append("final_conv")
NREP = int(os.environ.get("SDDM_REPEAT_N", "3"))
rows = {}
for d in sorted(glob.glob(os.path.join(REPO, "gpurun_out/abl_*_*"))):
    if not os.path.isdir(d):
        continue
    m = re.match(r".*/abl_(.+)_(\d+)$", d)
    op, fl = m.group(1), int(m.group(2))
    f = glob.glob(d + "/*kernel_trace.csv")
    if not f:
        continue
    k = [r for r in csv.DictReader(open(f[0])) if re.search(r"conv|final_kernel", r["Kernel_Name"])]
    k.sort(key=lambda r: int(r["Start_Timestamp"]))
    i = order.index(op)
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in k[i + 1:i + 1 + NREP]]
    rows.setdefault(op, {})[fl] = statistics.median(durs) if durs else float("nan")
names = {0: "full", 1: "-GNfin", 2: "-silu", 4: "-stage", 8: "-Kloop", 16: "-stats", 32: "-wload", 63: "-all"}
fls = sorted({f for v in rows.values() for f in v})
print("layer".ljust(18) + "".join(names.get(f, str(f)).rjust(9) for f in fls))
for op, v in rows.items():
    print(op.ljust(18) + "".join(f"{v.get(f, float('nan')):9.2f}" for f in fls))
