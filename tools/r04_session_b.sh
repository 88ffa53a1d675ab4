#!/bin/bash
# Round-4 session B: the query exchange, the division and atan2 variants timed (c3 and c3-descent,
# 128 steps per launch; nowqx = built without the exchange, WQX0 = the exchange's code with the
# identity mapping), c2 at lanes-per-env 2 / 8 / 16, then the bench lines (driver command,
# defaults, c4, c5) and the policy lanes-per-env sweep.
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
run f32shadow 300 python -u -m pytest tests/test_gpu_c3.py -k f32_handle -s -x --timeout 280 --timeout-method thread
PDENV_CELL_PIECES=0 run f32shadow_nopieces 300 python -u -m pytest tests/test_gpu_c3.py -k f32_handle -s -x --timeout 280 --timeout-method thread
for d in 0 1; do
  VARIANTS="base nowqx" FUSE=128 LAUNCHES=6 DESCENT=$d run exp_wqx_d$d 400 bash tools/exp_session.sh
  PDENV_WQX=0 FUSE=128 LAUNCHES=6 DESCENT=$d run exp_wqx0_d$d 200 python tools/time_fused.py
done
for l in 16 8 2; do
  N=4096 WIND=0 TILT=0 LPE=$l FUSE=128 LAUNCHES=6 run c2_lpe$l 200 python tools/time_fused.py
done
run benchdrv 600 python bench.py --steps 20 --warmup 5
run bench 600 python bench.py
for d in 0 1; do
  VARIANTS="base0 nomk noat" FUSE=128 LAUNCHES=6 DESCENT=$d run exp_div_atan2_d$d 600 bash tools/exp_session.sh
done
run c4 600 python bench.py --workload c4
run c5 600 python bench.py --workload c5
run plpe 600 python tools/policy_lpe_sweep.py
echo "=== done"
