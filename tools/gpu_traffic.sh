# HBM traffic per kernel launch: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (they cannot share a pass) over tools/profile_ops.py (B=16 x 16448, bf16, 2 reverse steps);
# tools/traffic.py maps the last step's dispatches onto the op list and writes profiles/<name>.json
# config #5 per GPU: OPS_ARGS="--batch 128 --num-samples 32832 --dtype f16 --lane-rows 64"
#   TRAFFIC_KEY="32832 128 f16" TRAFFIC_OUT=profiles/r04_config5_hbm_traffic.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/traffic_$c
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/traffic_$c -o run -- python3 tools/profile_ops.py --timesteps 2 ${OPS_ARGS} --json gpurun_out/traffic_ops_$c.json > gpurun_out/traffic_$c.log 2>&1 || { echo TRAFFIC_FAIL $c; tail -5 gpurun_out/traffic_$c.log; exit 1; }
done
python3 tools/traffic.py ${TRAFFIC_OUT:-profiles/r04_hbm_traffic.json} ${TRAFFIC_KEY} | cut -c1-600
echo TRAFFIC_OK
