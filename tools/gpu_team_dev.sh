# team-kernel iteration: its parity test, then per-layer profile + short bench with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS="tests/test_gpu_unet.py -k team" LOG=team_tests LIMIT=300 bash tools/gpu_tests.sh || exit 1
BENCH=1 bash tools/gpu_ab.sh "SDDM_TEAM=0" "" || exit 1
