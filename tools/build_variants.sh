#!/bin/bash
# Ablation builds of libpdenv for perf experiments (tools/sweep.py with PDENV_LIB=...).
cd "$(dirname "$0")/../psso-sac-for-powered-descent_amd"
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result -mllvm -disable-machine-licm"
for V in "$@"; do
  /opt/rocm/bin/hipcc $F -DPD_EXP_$V -o pdenv/libpdenv_$(echo $V | tr A-Z a-z).so csrc/pdenv.hip csrc/pdpso.hip &
done
wait
