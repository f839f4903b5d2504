# DiffWave (WORKLOAD=diffwave) or WaveGrad (WORKLOAD=wavegrad): GPU tests, bench, and the top
# kernels of a T=10 rocprofv3 --kernel-trace --stats run (per-shape table for WaveGrad).
#   WORKLOAD=wavegrad bash tools/gpu_spec.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
W=${WORKLOAD:-diffwave}
TF=tests/test_gpu_$W.py
timeout -k 10 300 python -u -m pytest $TF -x -q --timeout 200 --timeout-method thread > gpurun_out/${W}_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${W}_tests.log; exit 1; }
tail -1 gpurun_out/${W}_tests.log
timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline > gpurun_out/${W}_bench.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/${W}_bench.log; exit 1; }
tail -1 gpurun_out/${W}_bench.log | cut -c1-220
rm -rf gpurun_out/prof_$W
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$W -o run -- python3 bench.py --workload $W --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$W.log 2>&1 || { echo PROF_FAIL; tail -5 gpurun_out/prof_$W.log; exit 1; }
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_$W/run_kernel_stats.csv')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:8]: print(round(float(r['TotalDurationNs'])/1e6,3), r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:70])
"
[ "$W" = wavegrad ] && python3 tools/trace_shapes.py gpurun_out/prof_$W/run_kernel_trace.csv wg_
echo ALL_OK
