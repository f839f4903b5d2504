# WaveGrad: GPU tests, then kernel stats of a short sampling run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wavegrad.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/wg_tests.log; exit 1; }
tail -1 gpurun_out/wg_tests.log
rm -rf gpurun_out/prof_wg
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wg -o run -- python3 bench.py --workload wavegrad --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_wg.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/prof_wg.log; exit 1; }
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_wg/run_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total ms', tot/1e6)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:6]: print(round(float(r['TotalDurationNs'])/1e6,3), r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:70])
"
timeout -k 10 300 python3 bench.py --workload wavegrad --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/wg_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/wg_bench.log | cut -c1-160
echo ALL_OK
