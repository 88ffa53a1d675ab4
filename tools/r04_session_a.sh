#!/bin/bash
# Round-4 session A: device atan2 check, GPU tests + smoke on the Markstein / atan2_fd build, the
# division and atan2 variants timed against the round-3 arithmetic (c3 and c3-descent, 128 steps
# per launch), the bench lines, c4 and the policy-rollout lanes-per-env sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ "${PART:-1}" = 1 ]; then
run atan2 60 tools/bin/atan2_gpu_check
run gpu_tests 900 python -u -m pytest tests/ -m gpu --maxfail=6 -v --timeout 180 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
echo "=== done"
exit 0
fi
for d in 0 1; do
  VARIANTS="base nowqx base0 nomk noat" FUSE=128 LAUNCHES=6 DESCENT=$d run exp_div_atan2_d$d 600 bash tools/exp_session.sh
done
run benchdrv 600 python bench.py --steps 20 --warmup 5
run bench 600 python bench.py
run c4 600 python bench.py --workload c4
run plpe 600 python tools/policy_lpe_sweep.py
echo "=== done"
