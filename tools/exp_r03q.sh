#!/bin/bash
# Round-3 session q: lanes per env at 8 192 and 16 384 envs (with and without wind), completing
# session p's sweep for pd_create's default table, 128 env-steps per launch, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp LAUNCHES=4 FUSE=128
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03q.jsonl || exit $?; }
for r in 1 2; do
  for l in 2 4 8 16; do N=8192 LPE=$l run; done
  for l in 2 4 8 16; do N=8192 WIND=0 TILT=0 LPE=$l run; done
  for l in 2 4; do N=16384 WIND=0 TILT=0 LPE=$l run; done
done
echo done
