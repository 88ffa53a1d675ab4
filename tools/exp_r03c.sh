#!/bin/bash
# Round-3 session c: same-box A/B of this build against patched variants (tools/experiments):
# no_counts (counting compiled out), no_pair (one gust draw per sub-step), no_gust (no draws);
# c3 and c3-descent at FUSE 16, base also at 64; then counting runs (COUNT=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { timeout -k 10 180 python tools/time_fused.py >> gpurun_out/exp_r03c.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    for v in base no_counts no_pair no_gust; do
      lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
      PDENV_LIB=$lib DESCENT=$d run
    done
    FUSE=64 LAUNCHES=6 DESCENT=$d run
  done
done
DESCENT=0 COUNT=1 run
DESCENT=1 COUNT=1 run
echo done
