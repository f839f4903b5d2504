# round evidence: PMC traffic, headline bench (T=1000, CPU baseline), rocprofv3 kernel stats of the
# same workload (T=100), DiffWave and WaveGrad benches + kernel stats; the headline line carries the
# fp16 twin and fp32 as same-run variants; with CONFIG5=1 also config #5's PMC traffic and per-GPU bench.
# Usage: ROUND=r05 CONFIG5=1 bash tools/gpu_round_profiles.sh ; results land in gpurun_out/profiles/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r02}
O=gpurun_out/profiles
mkdir -p $O
# PMC traffic first, written where bench.py reads it, so the headline line carries it
TRAFFIC_OUT=profiles/${R}_hbm_traffic.json bash tools/gpu_traffic.sh || { echo TRAFFIC_FAIL; exit 1; }
cp profiles/${R}_hbm_traffic.json $O/
# the fp16 twin's traffic (the headline line's `variants.f16.roofline.traffic`)
OPS_ARGS="--dtype f16" TRAFFIC_KEY="16448 16 f16" TRAFFIC_OUT=profiles/${R}_f16_hbm_traffic.json bash tools/gpu_traffic.sh || { echo F16_TRAFFIC_FAIL; exit 1; }
cp profiles/${R}_f16_hbm_traffic.json $O/
timeout -k 10 900 python3 bench.py > $O/${R}_bench.json.log 2>&1 || { echo BENCH_FAIL; tail -5 $O/${R}_bench.json.log; exit 1; }
tail -1 $O/${R}_bench.json.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o run -- python3 bench.py --timesteps 100 --steps 1 --warmup 1 --no-cpu-baseline --no-variants > $O/${R}_bench_T100_rocprof.json.log 2>&1 || { echo PROF_FAIL; exit 1; }
cp gpurun_out/prof_bench/run_kernel_stats.csv $O/${R}_kernel_stats_T100_B16_bf16.csv
# (the fp16 twin and fp32 are the headline line's same-run `variants` since round 6)
if [ -n "$CONFIG5" ]; then   # config #5 per GPU: PMC traffic, then the bench line that reads it
  OPS_ARGS="--batch 128 --num-samples 32832 --dtype f16 --lane-rows 64" TRAFFIC_KEY="32832 128 f16" \
    TRAFFIC_OUT=profiles/${R}_config5_hbm_traffic.json bash tools/gpu_traffic.sh || { echo C5_TRAFFIC_FAIL; exit 1; }
  cp profiles/${R}_config5_hbm_traffic.json $O/
  timeout -k 10 900 python3 bench.py --batch 128 --num-samples 32832 --dtype f16 --no-cpu-baseline > $O/${R}_unet_config5_per_gpu_bench.json.log 2>&1 || { echo C5_FAIL; exit 1; }
  tail -1 $O/${R}_unet_config5_per_gpu_bench.json.log | cut -c1-200
fi
timeout -k 10 900 python3 bench.py --workload diffwave > $O/${R}_diffwave_bench.json.log 2>&1 || { echo DW_FAIL; tail -5 $O/${R}_diffwave_bench.json.log; exit 1; }
tail -1 $O/${R}_diffwave_bench.json.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dw -o run -- python3 bench.py --workload diffwave --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > $O/${R}_diffwave_T10_rocprof.json.log 2>&1 || { echo PROF_DW_FAIL; exit 1; }
cp gpurun_out/prof_dw/run_kernel_stats.csv $O/${R}_diffwave_kernel_stats_T10_B64_bf16.csv
timeout -k 10 900 python3 bench.py --workload wavegrad > $O/${R}_wavegrad_bench.json.log 2>&1 || { echo WG_FAIL; tail -5 $O/${R}_wavegrad_bench.json.log; exit 1; }
tail -1 $O/${R}_wavegrad_bench.json.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wg -o run -- python3 bench.py --workload wavegrad --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > $O/${R}_wavegrad_T10_rocprof.json.log 2>&1 || { echo PROF_WG_FAIL; exit 1; }
cp gpurun_out/prof_wg/run_kernel_stats.csv $O/${R}_wavegrad_kernel_stats_T10_B64_bf16.csv
echo ALL_OK
