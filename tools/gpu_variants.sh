# GPU parity tests, then the bench workload under several env settings ("VAR=val VAR2=val2" args)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/var$i.log 2>&1 || { echo VAR_FAIL $v; tail -5 gpurun_out/var$i.log; exit 1; }
  echo "$v => $(tail -1 gpurun_out/var$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "audio-s/s", d["ms_per_step"], "ms/step")')"
done
echo VAR_OK
