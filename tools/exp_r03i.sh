#!/bin/bash
# Round-3 session i: steps per launch 64 / 128 / 256 on c3 and c3-descent (the same 768 steps
# after burn-in), and what the profiler lists as available (PC sampling configurations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03i.jsonl || exit $?; }
for d in 0 1; do
  FUSE=64 LAUNCHES=12 DESCENT=$d run
  FUSE=128 LAUNCHES=6 DESCENT=$d run
  FUSE=256 LAUNCHES=3 DESCENT=$d run
done
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1 || true
echo done
