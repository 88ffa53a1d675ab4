#!/bin/bash
# Round-6 GPU sessions, in parts (PART=N), each under its own gpurun call.  Every GPU step runs
# under its own time limit; a crash, abort or time limit stops the part (no further GPU work).
#   1: the multi-rank product path (tests/test_gpu_multi_rank.py: c4 and c5 on two gloo ranks
#      sharing cuda:0, bit-identical to world 1), the GPU suite and the smoke on the build whose
#      step launches insert their own aero misses (no k_insert launch after each); the driver's
#      command and the fixed cost against the round-5 library (libpdenv_r05.so), interleaved;
#      the RCCL path of bench.py (torchrun, one rank, PD_BENCH_DIST=1: c3, c4, c5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PKG=psso-sac-for-powered-descent_amd/pdenv
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rccl() {  # name, args...
  local name=$1; shift
  PD_BENCH_DIST=1 run rccl_$name 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 "$@"
}
case "${PART:-1}" in
1)
  run gpu_multi 700 python -u -m pytest tests/test_gpu_multi_rank.py -x -v --timeout 600 --timeout-method thread
  run gpu_tests 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread --ignore tests/test_gpu_multi_rank.py
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for r in 1 2; do
    for v in r06 r05; do
      lib=$PKG/libpdenv.so; [ $v = r05 ] && lib=$PKG/libpdenv_r05.so
      PDENV_LIB=$lib run benchdrv_${v}_r$r 200 python bench.py --steps 20 --warmup 5 --secondary 0 --descent 0 --others 0 --cpu-baseline 0 --fresh 0
      for f in 20 128; do
        PDENV_LIB=$lib BURN=640 FUSE=$f LAUNCHES=6 run fix_${v}_f${f}_r$r 200 python tools/time_fused.py
      done
    done
  done
  rccl c3 --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --descent 0 --fresh 0 --others 0
  rccl c5 --workload c5 --steps 32 --warmup 8 --cpu-baseline 0
  rccl c4 --workload c4 --steps 4 --warmup 2 --cpu-baseline 0
  ;;
esac
echo "=== done"
