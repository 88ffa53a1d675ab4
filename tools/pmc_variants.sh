#!/bin/bash
# One rocprofv3 PMC pass (COUNTERS) over tools/time_fused.py for each library variant (VARIANTS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp LAUNCHES=${LAUNCHES:-8}
PKG=psso-sac-for-powered-descent_amd/pdenv
for v in ${VARIANTS:-base}; do
  lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
  PDENV_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $COUNTERS --output-format csv -d gpurun_out/pmcv_$v -o run -- python3 tools/time_fused.py > gpurun_out/pmcv_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "variant $v ok"
done
