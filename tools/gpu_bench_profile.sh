set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 300 python bench.py --timesteps 100 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_t100.log 2>&1 || { echo B100_FAIL; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 bench.py --timesteps 100 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
