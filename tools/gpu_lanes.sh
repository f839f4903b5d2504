# lane-split experiment: the B=16 headline with the batch split into concurrent lanes, with and
# without a phase offset between the lanes' streams
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 300 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/lanes.log 2>&1 || { echo FAIL "$1"; tail -20 gpurun_out/lanes.log; exit 1; }
  echo "$1: $(tail -1 gpurun_out/lanes.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run "SDDM_LANE_ROWS=16"
run "SDDM_LANE_ROWS=8"
run "SDDM_LANE_ROWS=8 SDDM_LANE_OFFSET_US=250"
run "SDDM_LANE_ROWS=8 SDDM_LANE_OFFSET_US=400"
run "SDDM_LANE_ROWS=8 SDDM_LANE_OFFSET_US=600"
run "SDDM_LANE_ROWS=4 SDDM_LANE_OFFSET_US=200"
echo ALL_OK
