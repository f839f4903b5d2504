# strip layers (levels 0-1) re-timed on the large K-streamed tiles (SDDM_NO_STRIP + forced cfg)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/svt
timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/svt/table.json > gpurun_out/svt/table.log 2>&1 || { echo FAIL_table; exit 1; }
for c in 0 1 2 3 12; do
SDDM_NO_TUNING=1 SDDM_NO_STRIP=1 SDDM_TILE_CFG=$c timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/svt/t$c.json > gpurun_out/svt/t$c.log 2>&1 || { echo FAIL_$c; tail -5 gpurun_out/svt/t$c.log; exit 1; }
echo "cfg $c: $(head -2 gpurun_out/svt/t$c.log | tail -1)"
done
echo ALL_OK
