# iteration check: UNet GPU parity tests, short bench, per-op profile, optional phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/it_tests.log; exit 1; }
tail -2 gpurun_out/it_tests.log
timeout -k 10 300 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/it_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/it_bench.log; exit 1; }
tail -1 gpurun_out/it_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench T=200:", d["value"], "audio-s/s", d["ms_per_step"], "ms")'
timeout -k 10 200 python tools/profile_ops.py > gpurun_out/it_ops.log 2>&1 || { echo OPS_FAIL; tail -20 gpurun_out/it_ops.log; exit 1; }
grep -v amdgpu.ids gpurun_out/it_ops.log | head -48
if [ -n "$STAMP_OPS" ]; then
timeout -k 10 200 python tools/stamps.py $STAMP_OPS > gpurun_out/it_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/it_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/it_stamps.log
fi
echo ALL_OK
