# full -m gpu suite (verbose; stops at the first failure) and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/gpu_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
