# rocprofv3 kernel stats of the spectrogram workloads (DiffWave config #3, WaveGrad config #4), short runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wg -o run -- python3 bench.py --workload wavegrad --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_wg.log 2>&1 || { echo PROF_WG_FAIL; tail -5 gpurun_out/prof_wg.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dw -o run -- python3 bench.py --workload diffwave --timesteps 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_dw.log 2>&1 || { echo PROF_DW_FAIL; tail -5 gpurun_out/prof_dw.log; exit 1; }
echo ALL_OK
