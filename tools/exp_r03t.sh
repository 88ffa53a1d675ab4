#!/bin/bash
# Round-3 session t: cell pieces with 3 exact terms instead of 4 (PD_CELL_EXACT=3, host and c3
# kernel objects, libpdenv_ex3.so; every piece within 5.6e-15 of sum |c phi|, 1 of 398 357 C_L
# pieces rejected): c3 and c3-descent at 128 env-steps per launch, base and variant, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FUSE=128 LAUNCHES=4
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03t.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    DESCENT=$d run
    PDENV_LIB=$PKG/libpdenv_ex3.so DESCENT=$d run
  done
done
echo done
