#!/bin/bash
# Round-3 session h: kernel arguments through a laundered kernarg pointer (SGPR spills 261 -> 137)
# against the pre-change kernel (tools/experiments/pre_kargs.patch): the c3/draws/parity GPU
# tests on this build, then c3 and c3-descent 64-step launches in alternating rounds, and this
# build at 128 steps per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_c3.py tests/test_gpu_draws.py tests/test_gpu_parity.py > gpurun_out/r03h_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r03h_tests.log
export LAUNCHES=6
run() { timeout -k 10 180 python tools/time_fused.py >> gpurun_out/exp_r03h.jsonl || exit $?; }
for r in 1 2; do
  for d in 0 1; do
    for v in base prek; do
      lib=$PKG/libpdenv.so; [ "$v" != base ] && lib=$PKG/libpdenv_$v.so
      FUSE=64 PDENV_LIB=$lib DESCENT=$d run
    done
  done
done
for d in 0 1; do FUSE=128 LAUNCHES=3 DESCENT=$d run; done
echo done
