# A/B of environment switches on the UNet per-layer profile (tools/profile_ops.py) and, with
# BENCH=1, on a short headline bench.  One variant per argument ("" = defaults):
#   bash tools/gpu_ab.sh "" "SDDM_XCD=0" "SDDM_STRIP_MPI=128 SDDM_STRIP_BLOCKS=512"
# OPS_ARGS passes extra profile_ops.py arguments (e.g. "--batch 8 --dtype f16").
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 150 python tools/profile_ops.py --timesteps ${OPS_T:-10} ${OPS_ARGS} --json gpurun_out/ab$i.json > gpurun_out/ab$i.log 2>&1 \
    || { echo "AB_FAIL [$v]"; tail -5 gpurun_out/ab$i.log; exit 1; }
  echo "[$v] $(head -2 gpurun_out/ab$i.log | tail -1)"
  if [ -n "$BENCH" ]; then
    env $v timeout -k 10 300 python bench.py --timesteps ${BENCH_T:-200} --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/ab${i}_bench.log 2>&1 \
      || { echo "AB_BENCH_FAIL [$v]"; tail -5 gpurun_out/ab${i}_bench.log; exit 1; }
    echo "   bench: $(tail -1 gpurun_out/ab${i}_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "audio-s/s", d["ms_per_step"], "ms/step")')"
  fi
done
echo AB_OK
