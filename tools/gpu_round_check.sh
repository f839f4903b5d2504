# round check: every -m gpu test (parity figures kept under gpurun_out/all.log), then the headline
# bench and the rocprofv3 kernel statistics of the same workload at T=100
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r04}
O=gpurun_out/profiles
mkdir -p $O
LOG=all LIMIT=900 bash tools/gpu_tests.sh || exit 1
cp gpurun_out/all.log $O/${R}_gpu_tests.log
timeout -k 10 900 python3 bench.py > $O/${R}_bench.json.log 2>&1 || { echo BENCH_FAIL; tail -5 $O/${R}_bench.json.log; exit 1; }
tail -1 $O/${R}_bench.json.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o run -- python3 bench.py --timesteps 100 --steps 1 --warmup 1 --no-cpu-baseline > $O/${R}_bench_T100_rocprof.json.log 2>&1 || { echo PROF_FAIL; exit 1; }
cp gpurun_out/prof_bench/run_kernel_stats.csv $O/${R}_kernel_stats_T100_B16_bf16.csv
echo ALL_OK
