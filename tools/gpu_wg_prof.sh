# WaveGrad: GPU tests, bench, and a per-shape kernel table from a T=10 rocprofv3 trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wavegrad.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -1 gpurun_out/wg_tests.log
timeout -k 10 240 python3 bench.py --workload wavegrad --no-cpu-baseline > gpurun_out/wg_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/wg_bench.log | cut -c1-200
rm -rf gpurun_out/prof_wg2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wg2 -o run -- python3 bench.py --workload wavegrad --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/wg_prof2.log 2>&1 || { echo PROF_FAIL; exit 1; }
python3 tools/trace_shapes.py gpurun_out/prof_wg2/run_kernel_trace.csv wg_
