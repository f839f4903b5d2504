# UNet round-end evidence on the final sources: PMC traffic (headline and config #5 geometry,
# written where bench.py reads them), the headline bench (T=1000, CPU baseline), its rocprofv3
# kernel statistics at T=100, and the config #5 per-GPU bench; results in gpurun_out/profiles/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r04}
O=gpurun_out/profiles
mkdir -p $O
TRAFFIC_OUT=profiles/${R}_hbm_traffic.json bash tools/gpu_traffic.sh || { echo TRAFFIC_FAIL; exit 1; }
OPS_ARGS="--batch 128 --num-samples 32832 --dtype f16 --lane-rows 64" TRAFFIC_KEY="32832 128 f16" TRAFFIC_OUT=profiles/${R}_config5_hbm_traffic.json bash tools/gpu_traffic.sh || { echo TRAFFIC5_FAIL; exit 1; }
cp profiles/${R}_hbm_traffic.json profiles/${R}_config5_hbm_traffic.json $O/
timeout -k 10 900 python3 bench.py > $O/${R}_bench.json.log 2>&1 || { echo BENCH_FAIL; tail -5 $O/${R}_bench.json.log; exit 1; }
tail -1 $O/${R}_bench.json.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o run -- python3 bench.py --timesteps 100 --steps 1 --warmup 1 --no-cpu-baseline > $O/${R}_bench_T100_rocprof.json.log 2>&1 || { echo PROF_FAIL; exit 1; }
cp gpurun_out/prof_bench/run_kernel_stats.csv $O/${R}_kernel_stats_T100_B16_bf16.csv
timeout -k 10 900 python3 bench.py --batch 128 --num-samples 32832 --dtype f16 --no-cpu-baseline > $O/${R}_unet_config5_per_gpu_bench.json.log 2>&1 || { echo C5_FAIL; exit 1; }
tail -1 $O/${R}_unet_config5_per_gpu_bench.json.log | cut -c1-200
echo ALL_OK
