# timing ablations of selected ops on the profiling build (tools/_stamps, SDDM_STAMPS_DBG bits:
# 2 no staging transform, 4 no input loads, 8 no MFMAs, 32 no weight DMA (tile), 64 no residual
# loads (strip)); one stamps.py run per flag set:
#   STAMP_OPS="ups.8.block1 downs.1.block2" FLAGS="0 4 8" bash tools/gpu_ablate.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for fl in ${FLAGS:-0}; do
  SDDM_STAMPS_DBG=$fl timeout -k 10 200 python tools/stamps.py $STAMP_OPS > gpurun_out/ablate_$fl.log 2>&1 || { echo ABLATE_FAIL $fl; tail -20 gpurun_out/ablate_$fl.log; exit 1; }
  echo "== flags $fl"
  grep -v amdgpu.ids gpurun_out/ablate_$fl.log
done
echo ALL_OK
