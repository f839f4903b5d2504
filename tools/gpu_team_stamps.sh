# per-op timeline of the team kernel (tools/team_stamps.py) at the bench geometry
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/team_stamps.py ${STAMP_ARGS} > gpurun_out/team_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/team_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/team_stamps.log
