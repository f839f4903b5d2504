# phase stamps of selected ops (profiling build tools/_stamps): STAMP_OPS="op1 op2 ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps.py $STAMP_OPS > gpurun_out/stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps.log
echo ALL_OK
