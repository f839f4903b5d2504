# per-layer ablation timing: kernel trace of a relaunched layer with ablation flags
# usage: gpu_ablate.sh "layer1 layer2" "0 1 2 8"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for op in $1; do for fl in $2; do
SDDM_NO_GRAPH=1 SDDM_REPEAT_OP=$op SDDM_REPEAT_N=3 SDDM_REPEAT_FLAGS=$fl timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/abl_${op}_$fl -o run -- python3 tools/profile_ops.py --timesteps 1 > gpurun_out/abl_${op}_$fl.log 2>&1 || { echo ABL_FAIL $op $fl; tail -5 gpurun_out/abl_${op}_$fl.log; exit 1; }
done; done
echo ABL_OK
