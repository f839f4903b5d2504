# round 3: conv_tile v2 (DMA-staged K pipeline) parity + per-layer timing against v1
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/tile2
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_long.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $D/tests.log; exit 1; }
tail -2 $D/tests.log
timeout -k 10 150 python tools/profile_ops.py --timesteps 10 --json $D/ops_v2.json > $D/ops_v2.log 2>&1 || { echo FAIL_v2; tail -20 $D/ops_v2.log; exit 1; }
SDDM_TILE_V1=1 timeout -k 10 150 python tools/profile_ops.py --timesteps 10 --json $D/ops_v1.json > $D/ops_v1.log 2>&1 || { echo FAIL_v1; tail -20 $D/ops_v1.log; exit 1; }
head -2 $D/ops_v1.log | tail -1
head -2 $D/ops_v2.log | tail -1
python - <<'PY'
import json
a = {o["name"]: o["avg_ms"] * 1e3 for o in json.load(open("gpurun_out/tile2/ops_v1.json"))}
b = {o["name"]: o["avg_ms"] * 1e3 for o in json.load(open("gpurun_out/tile2/ops_v2.json"))}
for k in a:
    if "tile" in k:
        print(f"{k:28s} v1 {a[k]:6.1f}  v2 {b[k]:6.1f}")
PY
for v in 0 1; do
SDDM_TILE_V1=$v timeout -k 10 200 python bench.py --timesteps 200 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $D/bench$v.log 2>&1 || { echo FAIL_bench$v; tail -20 $D/bench$v.log; exit 1; }
echo "TILE_V1=$v: $(tail -1 $D/bench$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo ALL_OK
