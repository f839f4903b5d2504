# per-layer timing of every conv_tile configuration (forced where it fits) and of conv_deep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/sweep/tests.log; exit 1; }
tail -1 gpurun_out/sweep/tests.log
export SDDM_NO_TUNING=1
SDDM_NO_TILE=1 timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/sweep/deep.json > gpurun_out/sweep/deep.log 2>&1 || { echo FAIL_deep; tail -5 gpurun_out/sweep/deep.log; exit 1; }
head -2 gpurun_out/sweep/deep.log | tail -1
timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/sweep/auto.json > gpurun_out/sweep/auto.log 2>&1 || { echo FAIL_auto; tail -5 gpurun_out/sweep/auto.log; exit 1; }
head -2 gpurun_out/sweep/auto.log | tail -1
for c in 0 1 2 3 4 5 6 7 8 9 10 11; do
SDDM_TILE_CFG=$c timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/sweep/t$c.json > gpurun_out/sweep/t$c.log 2>&1 || { echo FAIL_$c; tail -5 gpurun_out/sweep/t$c.log; exit 1; }
echo "cfg $c: $(head -2 gpurun_out/sweep/t$c.log | tail -1)"
done
for dc in 16:4:16 32:4:16 32:8:16 64:4:16 64:8:16 128:8:16 128:4:16 32:8:32 64:8:32 128:8:32 64:4:32 128:4:32 32:4:32; do
n=$(echo $dc | tr ':' '_')
SDDM_NO_TILE=1 SDDM_DEEP_CFG=$dc timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/sweep/d$n.json > gpurun_out/sweep/d$n.log 2>&1 || { echo FAIL_d$n; tail -5 gpurun_out/sweep/d$n.log; exit 1; }
echo "deep $dc: $(head -2 gpurun_out/sweep/d$n.log | tail -1)"
done
echo ALL_OK
