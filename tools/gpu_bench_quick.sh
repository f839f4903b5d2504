# short benches of the three workloads (profile + CPU baseline on the UNet line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --timesteps 100 --steps 2 --warmup 1 > gpurun_out/bq_unet.log 2>&1 || { echo UNET_FAIL; tail -20 gpurun_out/bq_unet.log; exit 1; }
tail -1 gpurun_out/bq_unet.log
timeout -k 10 300 python bench.py --workload diffwave --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bq_dw.log 2>&1 || { echo DW_FAIL; tail -20 gpurun_out/bq_dw.log; exit 1; }
tail -1 gpurun_out/bq_dw.log
timeout -k 10 300 python bench.py --workload wavegrad --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bq_wg.log 2>&1 || { echo WG_FAIL; tail -20 gpurun_out/bq_wg.log; exit 1; }
tail -1 gpurun_out/bq_wg.log
echo ALL_OK
