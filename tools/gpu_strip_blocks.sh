# strip-kernel grid target A/B (SDDM_STRIP_BLOCKS): per-layer launch times of the strip layers
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for nb in 256 128 512; do
SDDM_STRIP_BLOCKS=$nb timeout -k 10 120 python tools/profile_ops.py --timesteps 10 > gpurun_out/sb_$nb.log 2>&1 || { echo FAIL_$nb; tail -5 gpurun_out/sb_$nb.log; exit 1; }
echo "blocks $nb: $(grep per-step gpurun_out/sb_$nb.log)"
grep "strip" gpurun_out/sb_$nb.log | awk '{print "   ", $1, $NF}'
done
echo ALL_OK
