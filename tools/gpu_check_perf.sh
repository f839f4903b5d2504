# quick check after a kernel change: UNet GPU tests, per-layer table, short headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/unet_tests.log; exit 1; }
tail -1 gpurun_out/unet_tests.log
timeout -k 10 200 python tools/profile_ops.py --timesteps 10 --json gpurun_out/perlayer.json > gpurun_out/perlayer.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/perlayer.log; exit 1; }
timeout -k 10 300 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bq_unet.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bq_unet.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bq_unet.log').read().strip().splitlines()[-1]); print('T200 value', d['value'], 'ms/step', d['ms_per_step'], 'dominant', d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])"
echo ALL_OK
