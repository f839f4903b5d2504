# UNet GPU tests (verbose, per-test timeout) then the kernel sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/unet_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "PASS|FAIL|Error|error|rms" gpurun_out/unet_tests.log | tail -40; exit 1; }
grep -E "PASSED|FAILED|rms|lanes" gpurun_out/unet_tests.log | tail -40
bash tools/gpu_tile_sweep.sh
