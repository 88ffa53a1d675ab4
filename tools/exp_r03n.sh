#!/bin/bash
# Round-3 session n: the fine index (one word per sub-cell in place of the cell record) -- the
# parity / c3 shadow / draws GPU tests, then c3 and c3-descent at 128 env-steps per launch with
# and without it (PDENV_FINE=0), alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_draws.py > gpurun_out/r03n_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r03n_tests.log
export FUSE=128 LAUNCHES=4
run() { timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03n.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    DESCENT=$d run
    PDENV_FINE=0 DESCENT=$d run
  done
done
for d in 0 1; do PREC=f32 DESCENT=$d run; done
echo done
