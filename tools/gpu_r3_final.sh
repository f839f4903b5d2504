# round-end evidence after the last kernel-source change: full -m gpu suite + smoke, PMC traffic
# re-keyed to the current sources, headline bench and WaveGrad bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/profiles
mkdir -p $O
bash tools/gpu_r3_tests.sh || exit 1
TRAFFIC_OUT=profiles/r03_hbm_traffic.json bash tools/gpu_traffic.sh || { echo TRAFFIC_FAIL; exit 1; }
cp profiles/r03_hbm_traffic.json $O/
timeout -k 10 900 python3 bench.py > $O/r03_bench.json.log 2>&1 || { echo BENCH_FAIL; tail -5 $O/r03_bench.json.log; exit 1; }
tail -1 $O/r03_bench.json.log | cut -c1-160
timeout -k 10 300 python3 bench.py --workload wavegrad > $O/r03_wavegrad_bench.json.log 2>&1 || { echo WG_FAIL; exit 1; }
tail -1 $O/r03_wavegrad_bench.json.log | cut -c1-160
cp gpurun_out/prof_wg2/run_kernel_stats.csv $O/r03_wavegrad_kernel_stats_T10_B64_bf16.csv 2>/dev/null || true
echo ALL_OK
