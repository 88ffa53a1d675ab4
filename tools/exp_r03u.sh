#!/bin/bash
# Round-3 session u: (1) each lane's table view from an LDS copy staged once per workgroup
# (tools/experiments/lds_table_view.patch, libpdenv_tdesc.so: no lane-indexed global loads of
# the parameters at the head of every lookup; LPE-2 kernels 246 -> 233 VGPRs, the small-batch
# wind kernels' 28-52 B/lane scratch gone); (2) cell pieces with 3 exact terms (libpdenv_ex3.so).
# c3 shadow + parity GPU tests on tdesc, then c3 / c3-descent at 128 env-steps per launch for base,
# tdesc, ex3, and small wind batches (4 096 envs LPE 16, 8 192 LPE 8) for base / tdesc, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
PDENV_LIB=$PKG/libpdenv_tdesc.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_c3.py tests/test_gpu_parity.py > gpurun_out/r03u_tests.log 2>&1 || { tail -30 gpurun_out/r03u_tests.log; exit 1; }
tail -1 gpurun_out/r03u_tests.log
export FUSE=128 LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03u.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    DESCENT=$d run
    PDENV_LIB=$PKG/libpdenv_tdesc.so DESCENT=$d run
    PDENV_LIB=$PKG/libpdenv_ex3.so DESCENT=$d run
  done
  N=4096 run; PDENV_LIB=$PKG/libpdenv_tdesc.so N=4096 run
  N=8192 run; PDENV_LIB=$PKG/libpdenv_tdesc.so N=8192 run
done
echo done
