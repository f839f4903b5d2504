# round 3: per-layer kernel sweep at 8-row lanes, the merged table, then the B=16 headline as two
# concurrent 8-row lanes on that table (with and without a phase offset) against one 16-row lane
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/sweep8
mkdir -p $D
export SDDM_LANE_ROWS=8
P="timeout -k 10 120 python tools/profile_ops.py --batch 8 --timesteps 10"
SDDM_NO_TUNING=1 SDDM_NO_TILE=1 $P --json $D/deep.json > $D/deep.log 2>&1 || { echo FAIL_deep; tail -5 $D/deep.log; exit 1; }
SDDM_NO_TUNING=1 $P --json $D/auto.json > $D/auto.log 2>&1 || { echo FAIL_auto; tail -5 $D/auto.log; exit 1; }
for c in 0 1 2 3 4 5 6 7 8 9 10 11 12; do
SDDM_NO_TUNING=1 SDDM_TILE_CFG=$c $P --json $D/t$c.json > $D/t$c.log 2>&1 || { echo FAIL_$c; tail -5 $D/t$c.log; exit 1; }
done
for dc in 16:4:16 32:4:16 32:8:16 64:4:16 64:8:16 128:8:16 128:4:16 32:8:32 64:8:32 128:8:32 64:4:32 128:4:32 32:4:32; do
n=$(echo $dc | tr ':' '_')
SDDM_NO_TUNING=1 SDDM_NO_TILE=1 SDDM_DEEP_CFG=$dc $P --json $D/d$n.json > $D/d$n.log 2>&1 || { echo FAIL_d$n; tail -5 $D/d$n.log; exit 1; }
done
SWEEP_LANE_BATCH=8 python tools/sweep_merge.py $D $D/conv_tuning_b8.json | tail -3
SDDM_TUNING_FILE=$D/conv_tuning_b8.json $P --json $D/tuned.json > $D/tuned.log 2>&1 || { echo FAIL_tuned; tail -5 $D/tuned.log; exit 1; }
head -2 $D/tuned.log | tail -1
run() {
  env $1 timeout -k 10 200 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $D/lanes.log 2>&1 || { echo FAIL "$1"; tail -20 $D/lanes.log; exit 1; }
  echo "$1: $(tail -1 $D/lanes.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
unset SDDM_LANE_ROWS
run "SDDM_LANE_ROWS=16"
run "SDDM_LANE_ROWS=8 SDDM_TUNING_FILE=$D/conv_tuning_b8.json"
run "SDDM_LANE_ROWS=8 SDDM_TUNING_FILE=$D/conv_tuning_b8.json SDDM_LANE_OFFSET_US=300"
run "SDDM_LANE_ROWS=8 SDDM_TUNING_FILE=$D/conv_tuning_b8.json SDDM_LANE_OFFSET_US=150"
echo ALL_OK
