# SQ instruction / wait counters of the chain kernel (per dispatch), one --pmc pass per counter group
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_IFETCH SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_chain_$i
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_chain_$i -o run -- python3 tools/chain_stamps.py > gpurun_out/pmc_chain_$i.log 2>&1 || { echo PMC_FAIL $i; tail -3 gpurun_out/pmc_chain_$i.log; continue; }
  python3 - "$i" <<'PY'
import csv, glob, sys
i = sys.argv[1]
f = glob.glob(f"gpurun_out/pmc_chain_{i}/**/*counter_collection.csv", recursive=True)
if not f: print("no csv", i); sys.exit(0)
rows = [r for r in csv.DictReader(open(f[0])) if "conv_chain" in r.get("Kernel_Name", "")]
agg = {}
for r in rows:
    agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"  {k}: per dispatch {v[-1]:.4g} (dispatches {len(v)})")
PY
done
