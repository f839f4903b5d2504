# kernel trace of one sampling step with a layer relaunched back-to-back (I-cache / warm-up test)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for op in "$@"; do
SDDM_NO_GRAPH=1 SDDM_REPEAT_OP=$op SDDM_REPEAT_N=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rep_$op -o run -- python3 bench.py --timesteps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-profile > gpurun_out/rep_$op.log 2>&1 || { echo REP_FAIL; tail -5 gpurun_out/rep_$op.log; exit 1; }
done
echo REP_OK
