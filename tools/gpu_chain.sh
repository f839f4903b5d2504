# fused deep-level chain: GPU tests (chain vs per-layer, bench-batch forwards), per-op timing with
# the LDS plan printed, ablations of the chain kernel (SDDM_CHAIN_ABL bits: 1 no weight loads,
# 2 no staging, 4 no MFMAs), a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -x -v --timeout 200 --timeout-method thread -k "chain or bench_batch" > gpurun_out/chain_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASSED|FAILED|Error|error|assert|rms" gpurun_out/chain_tests.log | tail -30; exit 1; }
grep -E "passed|failed|rms" gpurun_out/chain_tests.log | tail -20
SDDM_CHAIN_DEBUG=1 timeout -k 10 300 python3 tools/profile_ops.py --timesteps 20 > gpurun_out/chain_ops.log 2>&1 || { echo OPS_FAIL; tail -5 gpurun_out/chain_ops.log; exit 1; }
head -60 gpurun_out/chain_ops.log
for ab in 1 2 4 7; do
  SDDM_CHAIN_ABL=$ab timeout -k 10 300 python3 tools/profile_ops.py --timesteps 20 > gpurun_out/chain_abl$ab.log 2>&1 || { echo ABL_FAIL $ab; tail -5 gpurun_out/chain_abl$ab.log; exit 1; }
  echo "ablation $ab: $(grep 'chain\[' gpurun_out/chain_abl$ab.log | head -1)"
done
timeout -k 10 300 python3 bench.py --timesteps 100 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/chain_bench.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/chain_bench.log; exit 1; }
tail -1 gpurun_out/chain_bench.log | cut -c1-300
