#!/bin/bash
# Round-3 session r: table-independent physics (sincos of alpha_eff/theta, grid-fin C_a, the
# inertia) computed inside the lookup's load latency (tools/experiments/pre_physics.patch,
# PD_EXP_PRE = 1 / 3 / 7): c3 shadow + parity GPU tests on the widest variant, then c3 and
# c3-descent at 128 env-steps per launch, base and variants, alternating, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
PDENV_LIB=$PKG/libpdenv_pre7.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_c3.py tests/test_gpu_parity.py > gpurun_out/r03r_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r03r_tests.log
export FUSE=128 LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03r.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    DESCENT=$d run
    for v in pre1 pre3 pre7; do PDENV_LIB=$PKG/libpdenv_$v.so DESCENT=$d run; done
  done
done
echo done
