# lane-split experiment: the B=16 headline with the batch split into concurrent lanes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lr in 16 8 4; do
  SDDM_LANE_ROWS=$lr timeout -k 10 300 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/lanes_$lr.log 2>&1 || { echo FAIL_$lr; tail -20 gpurun_out/lanes_$lr.log; exit 1; }
  echo "lanes $lr: $(tail -1 gpurun_out/lanes_$lr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo ALL_OK
