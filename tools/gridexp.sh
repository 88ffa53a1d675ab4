#!/bin/bash
# Interior grid resolution experiments (PDENV_GRID, grid sub-division builds libpdenv_subS.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { PDENV_LIB=$PKG/libpdenv$1.so PDENV_GRID=$2 PDENV_TAY_DEBUG=1 timeout -k 10 170 python tools/time_fused.py 2>&1 | grep -v amdgpu | sed "s/^{/{\"v\": \"$1 $2\", /" || exit 1; }
for r in 1 2; do
  for spec in ${SPECS:-"|"}; do run "${spec%%|*}" "${spec##*|}"; done
done
