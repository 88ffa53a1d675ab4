#!/bin/bash
# rocprofv3 PMC passes over the c3 fused workload (tools/time_fused.py), one pass per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp LAUNCHES=${LAUNCHES:-8}
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_p$i -o run -- python3 tools/time_fused.py > gpurun_out/pmc_p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok: $ctrs"
done <<< "${PASSES}"
