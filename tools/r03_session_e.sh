#!/bin/bash
# Round-3 session e: driver + parity GPU tests (c4 policy shadow, fused SAC step), then the c4/c5
# bench lines and their kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_drivers.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r03e_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c5 > gpurun_out/r03e_c5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --steps 32 --warmup 2 --cpu-baseline 0 > gpurun_out/r03e_c4.log 2>&1 || exit $?
grep '^{' gpurun_out/r03e_c5.log | cut -c1-400; grep '^{' gpurun_out/r03e_c4.log | cut -c1-400
STAGES="profc4 profc5" bash tools/gpu_session.sh
