# team-kernel ablations: per-op stamps with conv_deep dbg bits (1 no GN finalize, 2 no GN+SiLU,
# 4 no staging loads, 8 no K loop, 16 no stats, 32 no weight loads) set on every team op
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for d in ${ABL:-0 32 4 36}; do
  SDDM_TEAM_DBG=$d timeout -k 10 120 python tools/team_stamps.py > gpurun_out/team_abl_$d.log 2>&1 || { echo ABL_FAIL $d; tail -5 gpurun_out/team_abl_$d.log; exit 1; }
  echo "== dbg $d"; grep -v amdgpu.ids gpurun_out/team_abl_$d.log
done
