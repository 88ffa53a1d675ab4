#!/bin/bash
# Round-3 session j: cell pieces (binary64 interior queries from per-cell polynomials + 4 exact
# terms) -- the parity / c3 shadow / draws GPU tests, then c3 and c3-descent 64-step launches
# with and without the pieces (PDENV_CELL_PIECES=0) in alternating rounds, then 128 and 256
# steps per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_draws.py > gpurun_out/r03j_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r03j_tests.log
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03j.jsonl || exit $?; }
PDENV_TAY_DEBUG=1 FUSE=64 LAUNCHES=2 run 2> gpurun_out/r03j_debug.log
for r in 1 2; do
  for d in 0 1; do
    FUSE=64 LAUNCHES=6 DESCENT=$d run
    PDENV_CELL_PIECES=0 FUSE=64 LAUNCHES=6 DESCENT=$d run
  done
done
for d in 0 1; do
  FUSE=128 LAUNCHES=3 DESCENT=$d run
  FUSE=256 LAUNCHES=2 DESCENT=$d run
done
echo done
