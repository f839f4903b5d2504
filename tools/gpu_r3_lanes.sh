# round 3: per-layer profile at 16 and 8 rows, then the B=16 headline split into concurrent
# lanes of 8 rows with a phase offset between the lanes' streams
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 150 python tools/profile_ops.py --timesteps 10 --json gpurun_out/r3/ops16.json > gpurun_out/r3/ops16.log 2>&1 || { echo FAIL_ops16; tail -20 gpurun_out/r3/ops16.log; exit 1; }
head -1 gpurun_out/r3/ops16.log
SDDM_LANE_ROWS=8 timeout -k 10 150 python tools/profile_ops.py --batch 8 --timesteps 10 --json gpurun_out/r3/ops8.json > gpurun_out/r3/ops8.log 2>&1 || { echo FAIL_ops8; tail -20 gpurun_out/r3/ops8.log; exit 1; }
head -1 gpurun_out/r3/ops8.log
run() {
  env $1 timeout -k 10 200 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3/lanes.log 2>&1 || { echo FAIL "$1"; tail -20 gpurun_out/r3/lanes.log; exit 1; }
  echo "$1: $(tail -1 gpurun_out/r3/lanes.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run "SDDM_LANE_ROWS=16"
run "SDDM_LANE_ROWS=8"
run "SDDM_LANE_ROWS=8 SDDM_LANE_OFFSET_US=200"
run "SDDM_LANE_ROWS=8 SDDM_LANE_OFFSET_US=350"
run "SDDM_LANE_ROWS=8 SDDM_LANE_OFFSET_US=500"
run "SDDM_LANE_ROWS=4"
run "SDDM_LANE_ROWS=4 SDDM_LANE_OFFSET_US=150"
echo ALL_OK
