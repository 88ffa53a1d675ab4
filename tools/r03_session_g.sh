#!/bin/bash
# Round-3 session g: parity of the half-chunk last round (c3 shadow, device solve bit identity,
# fused == loop), then this build vs no_half (tools/experiments/no_half.patch) on c3 / c3-descent.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r03g_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03g_tests.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base no_half" bash tools/exp_r03f.sh
