#!/bin/bash
# Round-3 session m: early touch of the exact cell's piece (tools/experiments/piece_touch.patch)
# against this build, c3 and c3-descent at 128 env-steps per launch, alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FUSE=128 LAUNCHES=4
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03m.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    for v in base ${VARIANTS:-touch}; do
      lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
      PDENV_LIB=$lib DESCENT=$d run
    done
  done
done
echo done
