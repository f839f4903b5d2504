# GPU test runner: TESTS (default: tests) and extra pytest args ARGS; one pytest process, each test
# time-limited, verbose with -s so the printed parity figures land in the log.
# Usage: TESTS="tests/test_gpu_long.py" LOG=long bash tools/gpu_tests.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LOG=gpurun_out/${LOG:-gpu_tests}.log
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread ${ARGS} > $LOG 2>&1 \
  || { echo TESTS_FAIL; grep -E "PASSED|FAILED|Error|error|assert|rms" $LOG | tail -40; exit 1; }
grep -E "rms|passed|failed" $LOG | tail -40
