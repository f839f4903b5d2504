# DiffWave: GPU parity tests, then rocprofv3 kernel stats of a short config #3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_diffwave.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dw_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/dw_tests.log; exit 1; }
tail -1 gpurun_out/dw_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dw -o run -- python3 bench.py --workload diffwave --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_dw.log 2>&1 || { echo PROF_DW_FAIL; tail -5 gpurun_out/prof_dw.log; exit 1; }
tail -1 gpurun_out/prof_dw.log | cut -c1-400
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_dw/run_kernel_stats.csv")))
for r in rows[:8]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x {r['Calls']:>5}  {r['Percentage'][:5]}%  {r['Name'][:80]}")
PY
echo ALL_OK
