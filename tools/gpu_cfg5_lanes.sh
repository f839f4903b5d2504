# UNet GPU tests, short headline bench, config #5 per-GPU bench (B=128 x 32832, fp16, lanes of 64)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { echo TEST_FAIL; tail -20 gpurun_out/unet_tests.log; exit 1; }
grep -E "lane|config #5|passed" gpurun_out/unet_tests.log | tail -5
timeout -k 10 300 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/bq_unet.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bq_unet.log; exit 1; }
echo "headline T=200: $(tail -1 gpurun_out/bq_unet.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["lane_rows"])')"
timeout -k 10 300 python bench.py --batch 128 --num-samples 32832 --dtype f16 --timesteps 50 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/cfg5.log 2>&1 || { echo FAIL_cfg5; tail -5 gpurun_out/cfg5.log; exit 1; }
echo "config5 T=50: $(tail -1 gpurun_out/cfg5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["lane_rows"])')"
echo ALL_OK
