# HBM traffic of one sampling step per kernel: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# --pmc passes (they cannot share a pass), over tools/profile_ops.py --timesteps 1 (B=16, bf16)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/traffic_$c -o run -- python3 tools/profile_ops.py --timesteps 1 > gpurun_out/traffic_$c.log 2>&1 || { echo TRAFFIC_FAIL $c; tail -5 gpurun_out/traffic_$c.log; exit 1; }
done
echo TRAFFIC_OK
