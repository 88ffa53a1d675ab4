#!/bin/bash
# rocprofv3 PMC passes over tools/time_fused.py at bench.py's launch shape (FUSE env-steps per
# launch, default 128, LAUNCHES timed launches after the warmup), c3 and c3-descent: HBM traffic
# (FETCH_SIZE, WRITE_SIZE: separate passes) and the k_step instruction mix.  One counter set per
# run (gfx950 slot limits).  Output: gpurun_out/pmcF_<wl>_<pass>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FUSE=${FUSE:-128} LAUNCHES=${LAUNCHES:-3}
for d in 0 1; do
  wl=c3; [ $d = 1 ] && wl=desc
  i=0
  for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
              "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
              "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    DESCENT=$d timeout -s KILL 150 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmcF_${wl}_p$i -o run -- python3 tools/time_fused.py > gpurun_out/pmcF_${wl}_p$i.log 2>&1 || { echo "pass $wl $i failed rc=$?"; tail -3 gpurun_out/pmcF_${wl}_p$i.log; exit 1; }
    echo "pass $wl $i ok"
  done
done
