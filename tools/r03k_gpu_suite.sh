#!/bin/bash
# Round-3 session k: the whole -m gpu suite on the cell-piece build, the smoke, and a default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03k_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r03k_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03k_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r03k_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r03k_bench.log
echo done
