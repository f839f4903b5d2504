# per-layer timing of every conv_tile configuration (forced where it fits) and of conv_deep.
# SWEEP_OPS_ARGS: extra profile_ops.py arguments (config #5: "--batch 128 --num-samples 32832
# --dtype f16 --lane-rows 64"); SWEEP_DIR: output directory; SWEEP_NO_TESTS=1 skips the GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
SD=${SWEEP_DIR:-gpurun_out/sweep}
mkdir -p $SD
if [ -z "$SWEEP_NO_TESTS" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > $SD/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $SD/tests.log; exit 1; }
tail -1 $SD/tests.log
fi
export SDDM_NO_TUNING=1
SDDM_NO_TILE=1 timeout -k 10 120 python tools/profile_ops.py --timesteps 10 $SWEEP_OPS_ARGS --json $SD/deep.json > $SD/deep.log 2>&1 || { echo FAIL_deep; tail -5 $SD/deep.log; exit 1; }
head -2 $SD/deep.log | tail -1
timeout -k 10 120 python tools/profile_ops.py --timesteps 10 $SWEEP_OPS_ARGS --json $SD/auto.json > $SD/auto.log 2>&1 || { echo FAIL_auto; tail -5 $SD/auto.log; exit 1; }
head -2 $SD/auto.log | tail -1
for c in ${SWEEP_TILE_CFGS:-0 1 2 3 4 5 6 7 8 9 10 11 12}; do
SDDM_TILE_CFG=$c timeout -k 10 120 python tools/profile_ops.py --timesteps 10 $SWEEP_OPS_ARGS --json $SD/t$c.json > $SD/t$c.log 2>&1 || { echo FAIL_$c; tail -5 $SD/t$c.log; exit 1; }
echo "cfg $c: $(head -2 $SD/t$c.log | tail -1)"
done
for dc in ${SWEEP_DEEP_CFGS:-16:4:16 32:4:16 32:8:16 64:4:16 64:8:16 128:8:16 128:4:16 32:8:32 64:8:32 128:8:32 64:4:32 128:4:32 32:4:32 32:4:64 64:4:64 32:8:64}; do
n=$(echo $dc | tr ':' '_')
SDDM_NO_TILE=1 SDDM_DEEP_CFG=$dc timeout -k 10 120 python tools/profile_ops.py --timesteps 10 $SWEEP_OPS_ARGS --json $SD/d$n.json > $SD/d$n.log 2>&1 || { echo FAIL_d$n; tail -5 $SD/d$n.log; exit 1; }
echo "deep $dc: $(head -2 $SD/d$n.log | tail -1)"
done
echo ALL_OK
