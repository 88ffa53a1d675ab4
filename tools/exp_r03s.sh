#!/bin/bash
# Round-3 session s: clamped-line queries through the edge sub-cells' pieces (kFineLine, in the
# product library; PDENV_LINE_PIECES=0 restores the Taylor pieces): the full -m gpu suite, then
# c3 and c3-descent at 128 env-steps per launch with and without, alternating, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03s_tests.log 2>&1 || { tail -30 gpurun_out/r03s_tests.log; exit 1; }
tail -1 gpurun_out/r03s_tests.log
export FUSE=128 LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03s.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    DESCENT=$d run
    PDENV_LINE_PIECES=0 DESCENT=$d run
  done
done
echo done
