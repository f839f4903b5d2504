# A/B of the XCD-aware block order of the conv kernels: per-layer launch times with and without
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/xcd_on.json > gpurun_out/xcd_on.log 2>&1 || { echo FAIL_on; exit 1; }
SDDM_XCD=0 timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/xcd_off.json > gpurun_out/xcd_off.log 2>&1 || { echo FAIL_off; exit 1; }
timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/xcd_on2.json > gpurun_out/xcd_on2.log 2>&1 || { echo FAIL_on2; exit 1; }
SDDM_XCD=0 timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/xcd_off2.json > gpurun_out/xcd_off2.log 2>&1 || { echo FAIL_off2; exit 1; }
head -2 gpurun_out/xcd_on.log | tail -1; head -2 gpurun_out/xcd_off.log | tail -1; head -2 gpurun_out/xcd_on2.log | tail -1; head -2 gpurun_out/xcd_off2.log | tail -1
echo ALL_OK
