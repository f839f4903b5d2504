# DiffWave layer kernel A/B: weights held in registers (default) vs per-K-step loads (SDDM_DW_NOPRE)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in xcd plain; do
  if [ $v = plain ]; then export SDDM_DW_XCD=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dw_$v -o run -- python3 bench.py --workload diffwave --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_dw_$v.log 2>&1 || { echo PROF_FAIL $v; tail -5 gpurun_out/prof_dw_$v.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_dw_$v/run_kernel_stats.csv')):
    if 'dw_layer' in r['Name']: print('$v', float(r['AverageNs'])/1e3, 'us', r['Calls'])
"
done
echo ALL_OK
