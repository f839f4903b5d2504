# per-layer times under each forced conv_deep configuration (SDDM_DEEP_CFG=mt:nw)
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in default 32:4 64:4 128:4 32:8 64:8 128:8; do
  if [ $cfg = default ]; then unset SDDM_DEEP_CFG; else export SDDM_DEEP_CFG=$cfg; fi
  timeout -k 10 200 python tools/profile_ops.py --timesteps 5 > gpurun_out/cfg_${cfg/:/_}.log 2>&1 || { echo CFG_FAIL $cfg; tail -5 gpurun_out/cfg_${cfg/:/_}.log; exit 1; }
done
echo CFG_OK
