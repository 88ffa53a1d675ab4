#!/bin/bash
# rocprofv3 PMC passes over tools/time_fused.py (c3 and c3-descent, 16-step launches), one counter
# set per run (gfx950 slot limits: <= 8 SQ, <= 4 TCC counters per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp LAUNCHES=${LAUNCHES:-8}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P3="TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
for d in 0 1; do
  i=0
  for ctrs in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    DESCENT=$d timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc3_d${d}_p$i -o run -- python3 tools/time_fused.py > gpurun_out/pmc3_d${d}_p$i.log 2>&1 || { echo "pass d$d p$i failed rc=$?"; tail -5 gpurun_out/pmc3_d${d}_p$i.log; exit 1; }
    echo "pass d$d p$i ok"
  done
done
