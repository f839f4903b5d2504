# per-op timestamps inside the fused chain (normal build), plus ablation variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/chain_stamps.py > gpurun_out/chain_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -5 gpurun_out/chain_stamps.log; exit 1; }
cat gpurun_out/chain_stamps.log | grep -v amdgpu.ids
for ab in 1 4 7; do
  SDDM_CHAIN_ABL=$ab timeout -k 10 200 python3 tools/chain_stamps.py > gpurun_out/chain_stamps_abl$ab.log 2>&1 || { echo STAMPS_FAIL $ab; tail -5 gpurun_out/chain_stamps_abl$ab.log; exit 1; }
  echo "== ablation $ab"; grep -v amdgpu.ids gpurun_out/chain_stamps_abl$ab.log | tail -16
done
