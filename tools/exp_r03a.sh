#!/bin/bash
# Round-3 experiments, one GPU call: counter cost (no_counts), gust draws (no_gust) on c3 and
# c3-descent, PDENV_FUSE 16/32/64, and the PC-sampling configurations rocprofv3 offers here.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
run() { timeout -k 10 180 python tools/time_fused.py >> gpurun_out/exp_r03a.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    for v in base no_counts no_gust; do
      lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
      PDENV_LIB=$lib DESCENT=$d run
    done
  done
done
for d in 0 1; do for f in 16 32 64; do FUSE=$f LAUNCHES=$((384 / f)) DESCENT=$d run; done; done
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_list.txt 2>&1 || echo "list rc=$?"
echo done
