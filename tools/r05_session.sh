#!/bin/bash
# Round-5 GPU sessions, in parts (PART=N), each under its own gpurun call.  Every GPU step runs
# under its own time limit; a crash, abort or time limit stops the part (no further GPU work).
#   1: the per-launch fixed cost of the c3 kernel (steady state after bench.py's 640-step burn-in,
#      F = 1 / 4 / 20 / 128 fused steps per launch; PD_STAMP section clocks at F = 20 and 128),
#      c4 at the config's whole swarm on one GPU (262 144 particles, live list on / off), and the
#      driver's command on the current build.
#   2: the GPU suite and the smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
case "${PART:-1}" in
1)
  run benchdrv 300 python bench.py --steps 20 --warmup 5
  for f in 20 128 4 1; do
    L=$(( f >= 20 ? 6 : 24 ))
    BURN=640 FUSE=$f LAUNCHES=$L run fix_f$f 200 python tools/time_fused.py
  done
  for f in 20 128; do
    STATS=1 BURN=640 FUSE=$f LAUNCHES=6 PDENV_LIB=$PKG/libpdenv_stamp.so run stamp_f$f 200 python tools/time_fused.py
  done
  PDENV_COMPACT=1 run c4_262k_list 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0
  PDENV_COMPACT=0 run c4_262k_nolist 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0
  ;;
2)
  # the ABI-9 build (launcher checks, two-step divisions where the divisor needs them, tuning and
  # table flags through the ABI): the GPU suite and the smoke
  run gpu_tests 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  ;;
esac
echo "=== done"
