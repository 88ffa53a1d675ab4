#!/bin/bash
# Round-5 PMC passes over tools/time_fused.py (one rocprofv3 run per counter set, each under its
# own time limit).  CASES: space-separated names, each "tag:DESCENT:TABLE_FLAGS[:LIB]"; every case
# runs FETCH_SIZE, WRITE_SIZE and TCC_HIT_sum/TCC_MISS_sum passes at FUSE steps per launch after the
# BURN-step burn-in.  tools/pmc_r05.py reduces them (the last LAUNCHES k_step dispatches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FUSE=${FUSE:-128} LAUNCHES=${LAUNCHES:-3} BURN=${BURN:-640}
for c in ${CASES}; do
  IFS=: read -r tag d flags lib <<< "$c"
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    pn=$(echo "$pass" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    out=gpurun_out/pmc5_${tag}_${pn}
    DESCENT=$d TABLE_FLAGS=$flags PDENV_LIB=${lib:-psso-sac-for-powered-descent_amd/pdenv/libpdenv.so} timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv \
      -d $out -o run -- python3 tools/time_fused.py > $out.log 2>&1 || { echo "case $c pass $pass failed rc=$?"; exit 1; }
    echo "case $c pass $pass ok"
  done
done
