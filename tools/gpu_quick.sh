# GPU tests + short bench + per-op profile (each step time-limited, stop at first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python tools/profile_ops.py > gpurun_out/ops.log 2>&1 || { echo OPS_FAIL; tail -20 gpurun_out/ops.log; exit 1; }
head -50 gpurun_out/ops.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
echo ALL_OK
