#!/bin/bash
# Round-3 measurement session: GPU tests, smoke, the bench line (defaults and the driver's
# --steps 20 --warmup 5), rocprofv3 kernel traces of both (+ c4, c5), PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="${STAGES:-tests smoke bench benchdrv prof profdrv profc4 profc5}" bash tools/gpu_session.sh || exit $?
[ -n "$PMC" ] && bash tools/pmc_r03b.sh
echo finished
