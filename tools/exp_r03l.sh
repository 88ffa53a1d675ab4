#!/bin/bash
# Round-3 session l: where the cell-piece kernel's time goes -- PD_STAMP sections (c3, c3-descent)
# and one PMC pass of stall / issue counters each, at 128 env-steps per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp FUSE=128 LAUNCHES=3
PKG=psso-sac-for-powered-descent_amd/pdenv
for d in 0 1; do
  STATS=1 DESCENT=$d PDENV_LIB=$PKG/libpdenv_stamp.so timeout -k 10 240 python tools/time_fused.py >> gpurun_out/exp_r03l.jsonl || exit $?
done
for d in 0 1; do
  wl=c3; [ $d = 1 ] && wl=desc
  DESCENT=$d timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcl_${wl}_p1 -o run -- python3 tools/time_fused.py > gpurun_out/pmcl_${wl}_p1.log 2>&1 || { echo "pmc $wl failed"; exit 1; }
  DESCENT=$d timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcl_${wl}_p2 -o run -- python3 tools/time_fused.py > gpurun_out/pmcl_${wl}_p2.log 2>&1 || { echo "pmc $wl failed"; exit 1; }
  DESCENT=$d timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcl_${wl}_p3 -o run -- python3 tools/time_fused.py > gpurun_out/pmcl_${wl}_p3.log 2>&1 || { echo "pmc $wl failed"; exit 1; }
  echo "pmc $wl ok"
done
echo done
