set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python tools/profile_ops.py > gpurun_out/ops.log 2>&1 || { echo OPS_FAIL; exit 1; }
head -40 gpurun_out/ops.log
