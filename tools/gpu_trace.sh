# rocprofv3 kernel trace of the graph-replayed bench (no event profiling): per-kernel durations and gaps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/trace -o run -- python3 bench.py --timesteps ${TRACE_T:-20} --steps 1 --warmup 1 --no-cpu-baseline --no-profile ${TRACE_ARGS} > gpurun_out/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 gpurun_out/trace.log; exit 1; }
tail -1 gpurun_out/trace.log
find gpurun_out/trace -name "*.csv" | head
echo ALL_OK
