# PMC counters (per-dispatch averages, grouped by kernel name and grid) of one workload:
#   WORKLOAD=diffwave FILTER=dw_layer bash tools/gpu_pmc_kernels.sh          (bench.py --workload, T=2)
#   CMD="tools/profile_ops.py --timesteps 2" FILTER=conv_deep bash tools/gpu_pmc_kernels.sh
# one --pmc pass per counter group (PMC_GROUPS: ';'-separated; FETCH_SIZE and WRITE_SIZE in passes of their own)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
W=${WORKLOAD:-diffwave}
F=${FILTER:-dw_layer}
C=${CMD:-bench.py --workload $W --timesteps 2 --steps 1 --warmup 0 --no-cpu-baseline}
G=${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM;SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE}
TAG=${TAG:-$W}
i=0
IFS=';' read -ra GRPS <<< "$G"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  d=gpurun_out/pmc_${TAG}_$i
  rm -rf $d
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 $C > $d.log 2>&1 || { echo PMC_FAIL $i; tail -3 $d.log; exit 1; }
  python3 - "$d" "$F" <<'PY'
import csv, glob, sys, collections
d, filt = sys.argv[1], sys.argv[2]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
if not f: print("no csv", d); sys.exit(0)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if filt not in r.get("Kernel_Name", ""): continue
    key = (r["Kernel_Name"][:64], r.get("Grid_Size", r.get("Grid_Size_X", "")), r["Counter_Name"])
    agg[key].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"  {k[0]} grid {k[1]} {k[2]}: mean {sum(v)/len(v):.4g} (dispatches {len(v)})")
PY
done
