#!/bin/bash
# Time libpdenv variants (tools/variants.py) on the c3 fused workload, two alternating rounds.
# VARIANTS="base norbf ..." (base = the in-tree library); LPES="1 2 4" extra lanes-per-env runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PKG=psso-sac-for-powered-descent_amd/pdenv
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
    PDENV_LIB=$lib timeout -k 10 120 python tools/time_fused.py || exit $?
  done
  for l in ${LPES:-}; do
    LPE=$l timeout -k 10 120 python tools/time_fused.py | sed "s/^{/{\"lpe\": $l, /" || exit $?
  done
done
