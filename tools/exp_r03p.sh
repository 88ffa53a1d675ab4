#!/bin/bash
# Round-3 session p: lanes per env below 65 536 envs, on the current kernels (the default table
# in pd_create dates from round 1, before the LPE-2-only Taylor lines, cell pieces and fine
# index): c2 (4 096 envs, no wind, no tilt; reference integrator and RK4) and 16 384 / 32 768
# envs with wind, at each LPE, 128 env-steps per launch (RK4: 32), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03p.jsonl || exit $?; }
for r in 1 2; do
  for l in 2 16; do
    N=4096 WIND=0 TILT=0 FUSE=128 LPE=$l run
    N=4096 WIND=0 TILT=0 FUSE=32 INTEG=rk4 LPE=$l run
  done
  for l in 2 4 8; do N=16384 FUSE=128 LPE=$l run; done
  for l in 2 4; do N=32768 FUSE=128 LPE=$l run; done
  for l in 2 8 16; do N=4096 FUSE=128 LPE=$l run; done
done
echo done
