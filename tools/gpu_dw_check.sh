# DiffWave: GPU tests, then kernel stats of a short sampling run and a T=200 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_diffwave.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dw_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/dw_tests.log; exit 1; }
tail -1 gpurun_out/dw_tests.log
rm -rf gpurun_out/prof_dwc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dwc -o run -- python3 bench.py --workload diffwave --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_dwc.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/prof_dwc.log; exit 1; }
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_dwc/run_kernel_stats.csv')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:5]: print(round(float(r['TotalDurationNs'])/1e6,3), r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:60])
"
timeout -k 10 300 python3 bench.py --workload diffwave --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/dw_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/dw_bench.log | cut -c1-140
echo ALL_OK
