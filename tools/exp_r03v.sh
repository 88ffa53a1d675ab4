#!/bin/bash
# Round-3 session v: the grid-fin C_a / C_n interval slopes tabulated in LDS at staging (the same
# division on the same operands: same bits; libpdenv_gfs.so, built then from a patch that is gone:
# the change was kept and is in the product source since round 3): c3 shadow +
# parity GPU tests on the variant, then c3 / c3-descent at 128 env-steps per launch, base and
# variant, two rounds.  (A record of the round-3 session; it cannot be re-run as is.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
PDENV_LIB=$PKG/libpdenv_gfs.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_c3.py tests/test_gpu_parity.py > gpurun_out/r03v_tests.log 2>&1 || { tail -30 gpurun_out/r03v_tests.log; exit 1; }
tail -1 gpurun_out/r03v_tests.log
export FUSE=128 LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03v.jsonl || exit $?; }
for r in 1 2 3; do
  for d in 0 1; do
    DESCENT=$d run
    PDENV_LIB=$PKG/libpdenv_gfs.so DESCENT=$d run
  done
done
echo done
