# UNet GPU tests, then the tuned per-op profile (final / conv_in lines) and a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -x -v --timeout 300 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASS|FAIL|Error|error|rms" gpurun_out/unet_tests.log | tail -40; exit 1; }
grep -cE "PASSED" gpurun_out/unet_tests.log
timeout -k 10 120 python tools/profile_ops.py --timesteps 10 --json gpurun_out/ops.json > gpurun_out/ops.log 2>&1 || { echo FAIL_ops; tail -5 gpurun_out/ops.log; exit 1; }
head -2 gpurun_out/ops.log | tail -1
grep -E "final|conv_in" gpurun_out/ops.log
timeout -k 10 300 python bench.py --timesteps 100 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || { echo FAIL_bench; tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log
echo ALL_OK
