#!/bin/bash
# Round-3 session o: the Taylor and cell pieces' loads issued together
# (tools/experiments/joint_piece_loads.patch, libpdenv_joint.so): the c3 shadow / parity GPU tests
# on the variant, then c3 and c3-descent at 128 env-steps per launch, base and variant, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
PDENV_LIB=$PKG/libpdenv_joint.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_c3.py tests/test_gpu_parity.py > gpurun_out/r03o_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r03o_tests.log
export FUSE=128 LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03o.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    DESCENT=$d run
    PDENV_LIB=$PKG/libpdenv_joint.so DESCENT=$d run
  done
done
echo done
