# iteration run: team parity test, reference-noise and long-loop parity tests, per-op team stamps
# (8- and 4-wave teams), per-layer profile + short bench with and without the team kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TESTS="tests/test_gpu_unet.py -k team" LOG=team_tests LIMIT=300 bash tools/gpu_tests.sh || exit 1
TESTS="tests/test_gpu_torch_noise.py tests/test_gpu_long.py" LOG=parity_tests LIMIT=400 bash tools/gpu_tests.sh || exit 1
SDDM_TEAM=1 SDDM_PLAN_DEBUG=1 bash tools/gpu_team_stamps.sh || exit 1
cp gpurun_out/team_stamps.log gpurun_out/team_stamps_nw8.log
BENCH=1 bash tools/gpu_ab.sh "SDDM_TEAM=0" "SDDM_TEAM=1" || exit 1
