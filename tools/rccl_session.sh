#!/bin/bash
# The RCCL path of bench.py on one GPU: torchrun with one rank and PD_BENCH_DIST=1, so the nccl
# (= RCCL) process group is created and every collective of c3 (barrier, max-reduce), c4
# (subswarm all_gather) and c5 (all_gather_into_tensor of the transition slabs) runs on hardware.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PD_BENCH_DIST=1
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 1 "$@" > gpurun_out/rccl_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 gpurun_out/rccl_$name.log
  [ $rc -eq 0 ] || exit $rc
}
run c3 --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0
run c5 --workload c5 --steps 32 --warmup 8
run c4 --workload c4 --steps 2 --warmup 1 --cpu-baseline 0
