#!/bin/bash
# Round-3 session f: cost of one more dependent lookup load (tools/experiments/extra_*_level.patch)
# against this build, c3 and c3-descent, 64-step launches, two alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FUSE=64 LAUNCHES=6
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { timeout -k 10 180 python tools/time_fused.py >> gpurun_out/exp_r03f.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    for v in ${VARIANTS:-base extra_sub extra_cell}; do
      lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
      PDENV_LIB=$lib DESCENT=$d run
    done
  done
done
echo done
