# chain: parity tests, then per-op timestamps (normal and with weights / staging / MFMAs ablated)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -x -v --timeout 200 --timeout-method thread -k "chain or bench_batch" > gpurun_out/chain_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASSED|FAILED|Error|error|assert|rms" gpurun_out/chain_tests.log | tail -30; exit 1; }
grep -E "passed|failed|rms" gpurun_out/chain_tests.log | tail -12
timeout -k 10 200 python3 tools/chain_stamps.py > gpurun_out/chain_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -5 gpurun_out/chain_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_stamps.log
for ab in ${ABL:-4 7}; do
  SDDM_CHAIN_ABL=$ab timeout -k 10 200 python3 tools/chain_stamps.py > gpurun_out/chain_stamps_abl$ab.log 2>&1 || { echo STAMPS_FAIL $ab; tail -5 gpurun_out/chain_stamps_abl$ab.log; exit 1; }
  echo "== ablation $ab"; grep -v amdgpu.ids gpurun_out/chain_stamps_abl$ab.log | tail -16
done
