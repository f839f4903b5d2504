# tests, default bench, per-op profile and a rocprofv3 kernel-trace of a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python tools/profile_ops.py --json gpurun_out/ops.json > gpurun_out/ops.log 2>&1 || { echo OPS_FAIL; exit 1; }
head -12 gpurun_out/ops.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 bench.py --timesteps 100 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/prof.log; exit 1; }
echo ALL_OK
