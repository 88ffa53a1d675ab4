#!/bin/bash
# Round-6 GPU sessions, in parts (PART=N), each under its own gpurun call.  Every GPU step runs
# under its own time limit; a crash, abort or time limit stops the part (no further GPU work).
#   1: the multi-rank product path (tests/test_gpu_multi_rank.py: c4 and c5 on two gloo ranks
#      sharing cuda:0, bit-identical to world 1), the GPU suite and the smoke on the build whose
#      step launches insert their own aero misses (no k_insert launch after each); the driver's
#      command and the fixed cost against the round-5 library (libpdenv_r05.so), interleaved;
#      the RCCL path of bench.py (torchrun, one rank, PD_BENCH_DIST=1: c3, c4, c5).
#   2: the c4 / c5 traffic (tools/pmc_r06.sh: FETCH_SIZE, WRITE_SIZE, TCC hits of the policy and SAC
#      step launches at 32 768 / 262 144 particles and 4 096 envs); then a PC-sampling trial of the
#      c3 kernel (rocprofv3 --pc-sampling-beta-enabled, host_trap): where its issue slots go.
#      (The pool refuses PC sampling: that step never ran.)
#   3: non-temporal loads against L2 pollution, two interleaved rounds: the c4 actor weights
#      (libpdenv_pnt.so, tools/experiments/policy_nt.patch; c4 at 32 768 and 262 144 particles) and
#      the c3 fine-index word (libpdenv_fnt.so, fine_nt.patch; c3 and c3-descent); then the c2
#      lines (reference integrator with its CPU baseline, RK4) and the c5 line.
#   4: the c3 kernel's instruction stream by class: two rocprofv3 --pmc passes
#      over tools/time_fused.py (F = 128, after the burn-in) for c3 and c3-descent -- VALU by type
#      (INT32, INT64, CVT, F32 classes; F64 from the committed mix) and SALU / SMEM / LDS / VMEM /
#      branch counts with the VALU lane utilisation (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU).
#   5: what the c3 kernel's cold code costs its hot path: variants without the info tap (notap.patch,
#      productisable as a no-tap instantiation), without the miss solve (nomiss) and without the
#      neighbourhood verification (noverify; both wrong on the queries that need them, timing
#      only): a PMC pass (VALU, SALU, cycles) and two interleaved timing rounds, c3 and c3-descent.
#   6: staggered starts in the c3 windows (bench.py --stagger 128, the c3_sync sub-line the
#      synchronized starts): the driver's command twice and the default line.
#   7: the final build, part 1: the GPU suite (the two-rank test included), the smoke, the bench
#      lines (default, the driver's command, c4 at 32 768 and 262 144 particles, c5, c2, c2 RK4)
#      and a two-rank gloo rehearsal of the c3 line with both ranks on the one GPU.
#   8: the final build, part 2: rocprofv3 kernel traces (default, driver command, c4, c5) and the
#      c3 / c3-descent PMC passes (tools/pmc_r03b.sh); tools/collect_r03.py r06 reduces both.
#   9: the c3 unit under other compiler flags (tools/variants.py: loop strength reduction off,
#      -O2, both, no vectorizers; a static sweep of the ISA picked them: 1 % fewer VALU
#      instructions and up to 7 fewer VGPRs): a PMC pass each and two interleaved timing rounds.
#  10: the policy actor's weights in chunks of four parameters (one 16-byte load per lane for four
#      parameters; k_wchunk before each rollout): the policy, PSO, compaction and c4 shadow tests,
#      then c4 at 32 768 and 262 144 particles against the previous library (libpdenv_base.so),
#      two interleaved rounds.
#  13: c2's shape (4 096 envs, no wind, no tilt) at 8 against 16 lanes per env, 1 and 128 steps per
#      launch, two interleaved rounds: does LPE 8 (cell pieces) run the step as fast as LPE 16
#      (split payload sums)?  (A 32-env SAC actor tile at LPE 8 would read the hidden weights half
#      as often.)
#  11: the final build (chunked actor), part 1: the GPU suite, the smoke, the bench lines; part 12
#      (part 2): the c4 / c5 PMC passes and the rocprofv3 traces again.
#  14: the PSO driver on the chunked copy (ABI 11: pd_pso_step_chunked writes the rollout's weight
#      layout, pd_rollout_policy_chunked skips k_wchunk): the PSO / policy / c4 / two-rank tests,
#      then tools/c4_chunked_ab.py (the chunked path against the plain copy, interleaved in one
#      process, swarms bit-identical) at 32 768 and 262 144 particles, and a kernel trace of it;
#      the update call alone: tools/pso_grid_ab.py.
#  15: the RCCL path again on the final build (torchrun, one rank, PD_BENCH_DIST=1: c4 with the
#      chunked swarm copy, c5, c3).
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
2)
  run pmc6 900 bash tools/pmc_r06.sh
  run avail 120 rocprofv3 -L
  FUSE=128 LAUNCHES=3 BURN=128 run pcs_c3 180 rocprofv3 --pc-sampling-beta-enabled 1 --pc-sampling-method host_trap \
      --pc-sampling-unit time --pc-sampling-interval 10 --output-format csv -d gpurun_out/pcs_c3 -o run -- python3 tools/time_fused.py
  ;;
3)
  for r in 1 2; do
    for v in base pnt; do
      lib=$PKG/libpdenv.so; [ $v != base ] && lib=$PKG/libpdenv_$v.so
      PDENV_LIB=$lib run c4_${v}_r$r 300 python bench.py --workload c4 --steps 8 --warmup 2 --cpu-baseline 0
      PDENV_LIB=$lib run c4big_${v}_r$r 300 python bench.py --workload c4 --particles 262144 --steps 4 --warmup 1 --cpu-baseline 0
    done
    for v in base fnt; do
      lib=$PKG/libpdenv.so; [ $v != base ] && lib=$PKG/libpdenv_$v.so
      for d in 0 1; do
        PDENV_LIB=$lib DESCENT=$d BURN=640 FUSE=128 LAUNCHES=6 run t3_${v}_d${d}_r$r 200 python tools/time_fused.py
      done
    done
  done
  run c2 300 python bench.py --workload c2
  run c2rk4 300 python bench.py --workload c2 --integrator rk4
  run c5 300 python bench.py --workload c5
  ;;
4)
  PA="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32"
  PB="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU"
  for d in 0 1; do
    for pass in a b; do
      cs=$PA; [ $pass = b ] && cs=$PB
      DESCENT=$d BURN=640 FUSE=128 LAUNCHES=3 run pmc6mix_${pass}_d$d 120 rocprofv3 --pmc $cs --output-format csv \
          -d gpurun_out/pmc6mix_${pass}_d$d -o run -- python3 tools/time_fused.py
    done
  done
  ;;
5)
  for v in base notap nomiss noverify; do
    lib=$PKG/libpdenv.so; [ $v != base ] && lib=$PKG/libpdenv_$v.so
    PDENV_LIB=$lib DESCENT=0 BURN=640 FUSE=128 LAUNCHES=3 run pmc5v_$v 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv \
        -d gpurun_out/pmc5v_$v -o run -- python3 tools/time_fused.py
  done
  for r in 1 2; do
    for v in base notap nomiss noverify; do
      lib=$PKG/libpdenv.so; [ $v != base ] && lib=$PKG/libpdenv_$v.so
      for d in 0 1; do
        PDENV_LIB=$lib DESCENT=$d BURN=640 FUSE=128 LAUNCHES=6 run t5_${v}_d${d}_r$r 200 python tools/time_fused.py
      done
    done
  done
  ;;
6)
  run benchdrv6a 400 python bench.py --steps 20 --warmup 5
  run benchdrv6b 400 python bench.py --steps 20 --warmup 5
  run bench6 400 python bench.py
  ;;
7)
  run gpu_tests 1200 python -u -m pytest tests/ -m gpu -x -q --timeout 600 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  run bench 400 python bench.py
  run benchdrv 400 python bench.py --steps 20 --warmup 5
  run c4 300 python bench.py --workload c4
  run c4_262k 300 python bench.py --workload c4 --particles 262144 --steps 8 --warmup 2
  run c5 300 python bench.py --workload c5
  run c2 300 python bench.py --workload c2
  run c2rk4 300 python bench.py --workload c2 --integrator rk4
  PD_BENCH_BACKEND=gloo run gloo2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 32 --warmup 8 --descent 0 --fresh 0 --staggered 0
  ;;
8)
  run gpu_ins 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "inserts_its_misses or device_solve"
  STAGES="prof profdrv profc4 profc5" run profs 900 bash tools/gpu_session.sh
  run pmc 600 bash tools/pmc_r03b.sh
  ;;
9)
  for v in base nolsr nolsro2 o2 novec; do
    lib=$PKG/libpdenv.so; [ $v != base ] && lib=$PKG/libpdenv_$v.so
    PDENV_LIB=$lib DESCENT=0 BURN=640 FUSE=128 LAUNCHES=3 run pmc9_$v 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU \
        SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv \
        -d gpurun_out/pmc9_$v -o run -- python3 tools/time_fused.py
  done
  for r in 1 2; do
    for v in base nolsr nolsro2 o2 novec; do
      lib=$PKG/libpdenv.so; [ $v != base ] && lib=$PKG/libpdenv_$v.so
      for d in 0 1; do
        PDENV_LIB=$lib DESCENT=$d BURN=640 FUSE=128 LAUNCHES=6 run t9_${v}_d${d}_r$r 200 python tools/time_fused.py
      done
    done
  done
  ;;
10)
  run gpu_pol 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py tests/test_gpu_multi_rank.py -x -q \
      --timeout 600 --timeout-method thread -k "policy or pso or compaction or c4 or rollout or swarm or two_ranks"
  for r in 1 2; do
    for v in new base; do
      lib=$PKG/libpdenv.so; [ $v = base ] && lib=$PKG/libpdenv_base.so
      PDENV_LIB=$lib run c4_${v}_r$r 300 python bench.py --workload c4 --steps 8 --warmup 2 --cpu-baseline 0
      PDENV_LIB=$lib run c4big_${v}_r$r 300 python bench.py --workload c4 --particles 262144 --steps 4 --warmup 1 --cpu-baseline 0
    done
  done
  ;;
11)
  PART=7 bash tools/r06_session.sh
  ;;
12)
  run pmc6 900 bash tools/pmc_r06.sh
  STAGES="prof profdrv profc4 profc5" run profs 900 bash tools/gpu_session.sh
  ;;
14)
  run gpu_chunk 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_drivers.py tests/test_gpu_multi_rank.py -x -q \
      --timeout 600 --timeout-method thread -k "policy or pso or compaction or c4 or rollout or swarm or two_ranks or chunked"
  P=32768 G=8 ROUNDS=6 run ab14_32k 300 python -u tools/c4_chunked_ab.py
  P=262144 G=4 ROUNDS=6 run ab14_262k 300 python -u tools/c4_chunked_ab.py
  P=262144 G=2 ROUNDS=2 run kt14 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt14 -o p -- \
      python3 -u tools/c4_chunked_ab.py
  P=262144 run grid14_262k 120 python -u tools/pso_grid_ab.py
  P=32768 ROUNDS=20 run grid14_32k 120 python -u tools/pso_grid_ab.py
  ;;
15)
  rccl c4 --workload c4 --steps 4 --warmup 2 --cpu-baseline 0
  rccl c5 --workload c5 --steps 32 --warmup 8 --cpu-baseline 0
  rccl c3 --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --descent 0 --fresh 0 --others 0
  ;;
13)
  for r in 1 2; do
    for l in 16 8; do
      for f in 128 1; do
        L=$(( f > 1 ? 6 : 60 ))
        N=4096 LPE=$l WIND=0 TILT=0 FUSE=$f LAUNCHES=$L BURN=256 run t13_l${l}_f${f}_r$r 200 python tools/time_fused.py
      done
    done
  done
  ;;
esac
echo "=== done"
