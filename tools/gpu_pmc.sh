# PMC counter passes (each its own rocprofv3 run; no tracing domains combined with --pmc)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc$i -o run -- python3 tools/profile_ops.py --timesteps 2 > gpurun_out/pmc$i.log 2>&1 || { echo PMC_FAIL $grp; tail -5 gpurun_out/pmc$i.log; exit 1; }
done
echo PMC_OK
