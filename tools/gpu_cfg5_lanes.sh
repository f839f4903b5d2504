# config #5 per-GPU plan (B=128 x 32832, fp16): UNet GPU tests, then lane size A/B at T=50
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { echo TEST_FAIL; tail -20 gpurun_out/unet_tests.log; exit 1; }
grep -E "rms|passed" gpurun_out/unet_tests.log | tail -8
for lr in 64 128; do
SDDM_LANE_ROWS=$lr timeout -k 10 300 python bench.py --batch 128 --num-samples 32832 --dtype f16 --timesteps 50 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/cfg5_$lr.log 2>&1 || { echo FAIL_$lr; tail -5 gpurun_out/cfg5_$lr.log; exit 1; }
echo "lane_rows $lr: $(tail -1 gpurun_out/cfg5_$lr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo ALL_OK
