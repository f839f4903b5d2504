# round-4 batch: WaveGrad check, final-kernel frame-tile A/B, strip phase stamps, then the round check
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
WORKLOAD=wavegrad bash tools/gpu_spec.sh || exit 1
BENCH=1 bash tools/gpu_ab.sh "" "SDDM_FINAL_FT=16" || exit 1
STAMP_OPS="downs.1.block2 downs.3.block2 ups.12.block1 ups.10 ups.14.block1" bash tools/gpu_stamps.sh || exit 1
ROUND=${ROUND:-r04_base} bash tools/gpu_round_check.sh || exit 1
