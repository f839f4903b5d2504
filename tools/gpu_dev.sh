# dev loop: GPU parity tests, per-op profile, phase stamps of selected ops (args)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python tools/profile_ops.py > gpurun_out/ops.log 2>&1 || { echo OPS_FAIL; tail -20 gpurun_out/ops.log; exit 1; }
head -50 gpurun_out/ops.log
if [ $# -gt 0 ]; then timeout -k 10 300 python tools/stamps.py "$@" > gpurun_out/stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/stamps.log; exit 1; }; cat gpurun_out/stamps.log; fi
echo DEV_OK
