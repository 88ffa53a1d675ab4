#!/bin/bash
# Round-6 PMC passes over the c4 and c5 bench commands (one rocprofv3 run per counter set, each
# under its own time limit): FETCH_SIZE, WRITE_SIZE and TCC_HIT_sum/TCC_MISS_sum of the k_step
# launches.  tools/pmc_r06.py reduces them to bytes per particle-episode / env-step
# (profiles/r06_pmc_c4c5.json, read by bench.py for roofline.traffic).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CASES=${CASES:-"c4_32768 c4_262144 c5"}
for c in $CASES; do
  case $c in
    c4_32768) args="--workload c4 --particles 32768 --steps 4 --warmup 2 --cpu-baseline 0" ;;
    c4_262144) args="--workload c4 --particles 262144 --steps 2 --warmup 1 --cpu-baseline 0" ;;
    c5) args="--workload c5 --steps 64 --warmup 8 --cpu-baseline 0" ;;
  esac
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    pn=$(echo "$pass" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    out=gpurun_out/pmc6_${c}_${pn}
    timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $out -o run -- python3 bench.py $args \
      > $out.log 2>&1 || { echo "case $c pass $pass failed rc=$?"; exit 1; }
    echo "case $c pass $pass ok"
  done
done
