#!/bin/bash
# Round-3 session b: parity of the paired gust draws and flag-gated counters (c3 + draws + wind
# shadow tests), then time_fused: this build vs the counter-free round-2-style build
# (libpdenv_no_counts), c3 and c3-descent, FUSE 16 and 64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_draws.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { timeout -k 10 180 python tools/time_fused.py >> gpurun_out/exp_r03b.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    for f in 16 64; do
      FUSE=$f LAUNCHES=$((384 / f)) DESCENT=$d run
      PDENV_LIB=$PKG/libpdenv_no_counts.so FUSE=$f LAUNCHES=$((384 / f)) DESCENT=$d run
    done
  done
done
DESCENT=0 COUNT=1 run
DESCENT=1 COUNT=1 run
echo done
