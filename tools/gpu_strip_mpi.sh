# strip kernel A/B: pixels per iteration (SDDM_STRIP_MPI) x grid target (SDDM_STRIP_BLOCKS)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "256 256" "128 512" "128 256" "128 1024"; do
set -- $cfg
SDDM_STRIP_MPI=$1 SDDM_STRIP_BLOCKS=$2 timeout -k 10 120 python tools/profile_ops.py --timesteps 10 > gpurun_out/sm_$1_$2.log 2>&1 || { echo FAIL_$1_$2; tail -5 gpurun_out/sm_$1_$2.log; exit 1; }
echo "mpi $1 blocks $2: $(grep per-step gpurun_out/sm_$1_$2.log)"
grep "strip" gpurun_out/sm_$1_$2.log | awk '{print "   ", $1, $NF}'
done
echo ALL_OK
