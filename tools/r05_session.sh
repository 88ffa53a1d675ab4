#!/bin/bash
# Round-5 GPU sessions, in parts (PART=N), each under its own gpurun call.  Every GPU step runs
# under its own time limit; a crash, abort or time limit stops the part (no further GPU work).
#   1: the per-launch fixed cost of the c3 kernel (steady state after bench.py's 640-step burn-in,
#      F = 1 / 4 / 20 / 128 fused steps per launch; PD_STAMP section clocks at F = 20 and 128),
#      c4 at the config's whole swarm on one GPU (262 144 particles, live list on / off), and the
#      driver's command on the current build.
#   2: the GPU suite and the smoke.
#   3: the binary32 handle with the binary64 state chain: its tests and timing.
#   4: c3 / c3-descent traffic and time with and without the fine index (PMC passes).
#   5: the suite, smoke, fixed cost, driver command, c5 and c4-262k on the round-5 build.
#   6: the suite, smoke, c5 breakdown, fixed cost and driver command of the reordered prologue, then 4.
#   7: refill rollouts and the fused info tap: tests, c4 timings; the binary32 landing_burn diagnostic.
#   8: batched refill (slots handed particles once k of a wave's wait): tests, c4 timings per batch.
#   9: the auto batch (half a wave): tests, c4 at the whole swarm by default and at batches 12 / 24.
#  10: the suite and smoke on the refill / experiment-free build; SAC actor section clocks; c4 and
#      the driver's command.
#  11: SAC actor tile variants' section clocks (tools/mlp_clocks.hip over other tile versions).
#  12: the actor tile with whole-line weight fragments (v3): clocks against v1 (cold and warm),
#      the SAC tests, c5 and its breakdown.
#  13: v4 (layer 1 with the state width at compile time): clocks.
#  14: v4's hidden layer: fewer workgroups (shared L2 or per-CU bound?), tiles in flight, prefetch.
#  15: v5 (rotating fragment buffers behind scheduling barriers): clocks.
#  16: the hidden layer taken apart: loads only, loads beside independent MFMAs, v6 (A fragments
#      double-buffered from LDS).
#  17: loads only, the MFMA fragment pattern against 1 KB contiguous per wave load.
#  18: v7 (weights through a wave-private LDS ring by LDS DMA) against v5, with the heads checked
#      against a host forward pass.
#  19: v7's ring depth and tiles in flight.
#  20: v8 (the next block's fragments read from LDS during this block's MFMAs).
#  21: v8 taken apart: without the DMA, without the weight-fragment reads, without both.
#  22: v9 (whole-line loads into registers, swizzled into the LDS ring by the wave) against v7.
#  23: the product actor tile (v7: LDS DMA ring, layer 1 at compile-time width, head biases
#      early): the SAC tests, c5, its breakdown, the tile's clocks.
#  24: the staging loads issued ahead of the actor prologue: SAC tests, c5, breakdown, c3 fixed cost.
#  25: refill from the waves' own particle ranges: the compaction tests, c4 at the whole swarm by
#      own share and batch.
#  26: the round's measurement, part 1: the GPU suite, the smoke, the bench lines (default, the
#      driver's command, c4 at 32 768 and 262 144 particles, c5, c2).
#  27: part 2: rocprofv3 kernel traces (default, driver command, c4, c5) and the PMC passes
#      (tools/collect_r03.py r05 reduces both into profiles/).
#  28: the c3 kernel under other compiler scheduling strategies (tools/variants.py: max-memory-clause,
#      iterative-ilp, max-ilp, metric bias 0), c3 and c3-descent, two interleaved rounds.
#  29: refill rollouts in a given hand-out order (the previous generation's longest episodes first):
#      the compaction tests, c4 at the whole swarm with and without the order; then part 28.
#  30: where a 4 096-env launch's fixed cost goes (c5's shape without the actor: LPE 16, no wind):
#      PD_STAMP section clocks at 1 and 128 steps per launch.
#  31: parts 28 and 30 (part 29's run of 28 used a binding the variants did not export).
#  32: the build with the c3 unit scheduled for memory clauses: the c3 tests, c3 / c3-descent timing.
#  33: the final build: part 26 again (suite, smoke, bench lines); 34: part 27 again (traces, PMC).
#  35: more scheduler flags on top of max-memory-clause (clause length 32, the AMDGPU pressure
#      trackers, no high-pressure rescheduling) and max-ilp with trackers: c3 / c3-descent.
#  36: c4 at the config's 32 768 particles per GPU: refill (one launch, no live-count reads)
#      against the per-check launches, two rounds.
#  37: the actor tile's weight blocks requested one block ahead across tile groups and layers (the
#      first before layer 1): clocks, the SAC tests, c5.
#  38: refill by default for every windless swarm: the policy / PSO / compaction / c4 shadow tests,
#      c4 at 32 768 and 262 144 particles.
#  39 / 40: the final build: part 26 (suite, smoke, bench lines) and part 27 (traces, PMC) again.
#  41: the driver window's launch/sync gap: the driver's command (c3 only) with the host spinning
#      on completion (tools/spin_probe.py) and/or kernel arguments in device memory
#      (HIP_FORCE_DEV_KERNARG=1), three interleaved rounds.
#  42: c5 with and without the HIP graph (one pd_step_sac_fused launch per step either way), three
#      interleaved rounds, and a rocprofv3 kernel trace of each (the gaps between the step kernels).
#  43: eager c5 by default: the SAC / collector tests, bench.py --workload c5 (twice) and the
#      default line (with its other_workloads).
#  44: the c5 line with its kernel time from the timed region's events: twice, plus the rocprofv3
#      stats of the same command (the k_step<SAC> average to compare).
#  45: c4 with the subswarm membership mirrored on the host (a migration no longer reads the
#      device back) and pinned index copies: the PSO tests, c4 twice, the rocprofv3 trace.
#  46: part 45 again with share_information on the device (no read-back of the subswarm bests).
#  47: part 45 again: the share draws and the migration writes as kernel scalars (no host copies).
#  48: part 45 again: the best subswarm's row taken without indexing by a 0-d tensor (a read-back).
#  50: the final build again: part 26 (suite, smoke, bench lines).
#  51: part 45 again: the PSO update with four parameters per thread (one Philox draw, loads first).
#  49: part 45 again: the migration mirror and scalar writes kept, share_information back on the host
#      path (the device path measured no better: its ~25 small kernels cost what the read-back did).
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
case "${PART:-1}" in
1)
  run benchdrv 300 python bench.py --steps 20 --warmup 5
  for f in 20 128 4 1; do
    L=$(( f >= 20 ? 6 : 24 ))
    BURN=640 FUSE=$f LAUNCHES=$L run fix_f$f 200 python tools/time_fused.py
  done
  for f in 20 128; do
    STATS=1 BURN=640 FUSE=$f LAUNCHES=6 PDENV_LIB=$PKG/libpdenv_stamp.so run stamp_f$f 200 python tools/time_fused.py
  done
  # (the records of part 1 came from the pre-ABI-9 library, where the PDENV_COMPACT environment
  # switch chose the live list; ABI 9 removed every getenv switch, so the same comparison is now
  # made with the tuning flags below -- refill off, list on / off)
  run c4_262k_list 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0 --policy-list 1 --policy-refill 0
  run c4_262k_nolist 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0 --policy-list 0 --policy-refill 0
  ;;
2)
  # the ABI-9 build (launcher checks, two-step divisions where the divisor needs them, tuning and
  # table flags through the ABI): the GPU suite and the smoke
  run gpu_tests 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  ;;
3)
  # binary32 handles with the binary64 state chain: their tests (teacher-forced against the
  # reference on every channel, the c3 shadow at the fp32 tolerance, fused == per-step, device
  # solve, RK4), then c3 at F = 128 in both precisions
  run gpu_f32 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_rk4.py -m gpu -x -v \
      --timeout 300 --timeout-method thread -k "f32 or fused_equals or device_solve or rk4 or full_swarm or launcher" -s
  for p in f32 f64; do
    BURN=640 FUSE=128 LAUNCHES=6 PREC=$p run t_$p 200 python tools/time_fused.py
  done
  ;;
4)
  # where c3-descent's traffic comes from: the fine index against the cell / sub-cell records
  # (PD_TABLES_NO_FINE_INDEX = 2) and against the two-level index (libpdenv_idx2.so, built by
  # python tools/variants.py idx2=patch:tools/experiments/two_level_index.patch,-DPD_IDX2=1,host: a word per
  # cell, L2-resident, and the refined cells' sub-cell words), c3 and c3-descent: the variant's
  # bit-identity tests, PMC traffic + L2 hits, then the timing (two interleaved rounds)
  V=psso-sac-for-powered-descent_amd/pdenv/libpdenv_idx2.so
  PDENV_LIB=$V run idx2_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -m gpu -x -q \
      --timeout 300 --timeout-method thread -k "fine_index or c3_shadowed or cell_pieces"
  CASES="d_fine:1:0 d_rec:1:2 d_idx2:1:0:$V c_fine:0:0 c_idx2:0:0:$V" run pmc5 900 bash tools/pmc_r05.sh
  for r in 1 2; do
    for c in "1 0 base" "1 0 idx2" "0 0 base" "0 0 idx2" "1 2 base"; do
      set -- $c
      lib=psso-sac-for-powered-descent_amd/pdenv/libpdenv.so; [ "$3" = idx2 ] && lib=$V
      PDENV_LIB=$lib DESCENT=$1 TABLE_FLAGS=$2 BURN=640 FUSE=128 LAUNCHES=6 run t4_r${r}_d$1_f$2_$3 200 python tools/time_fused.py
    done
  done
  ;;
5)
  # the build with the binary64 state chain (binary32 handles), the SAC actor's latency plan and
  # the LDS tables staged from one image: the GPU suite (with the new f32 bounds, the launcher
  # checks and the full-swarm compaction test) and the smoke, then the per-launch fixed cost
  # (F = 1 / 20 / 128, binary64 and binary32), the driver's command, c5, c4 at the whole swarm
  run gpu_tests 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -s
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for f in 20 128 1; do
    L=$(( f >= 20 ? 6 : 24 ))
    BURN=640 FUSE=$f LAUNCHES=$L run fix5_f$f 200 python tools/time_fused.py
  done
  BURN=640 FUSE=128 LAUNCHES=6 PREC=f32 run t5_f32 200 python tools/time_fused.py
  run benchdrv5 300 python bench.py --steps 20 --warmup 5
  run c5_5 300 python bench.py --workload c5
  run c4_262k_5 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --policy-list 0
  ;;
6)
  # the build with the env state requested ahead of the table staging (and of the SAC actor):
  # the GPU suite and the smoke, the c5 breakdown, the fixed cost, the driver's command; then
  # part 4 (the index experiment)
  run gpu_tests 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -s
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  run c5_breakdown 300 python tools/c5_breakdown.py
  for f in 20 1; do
    L=$(( f >= 20 ? 6 : 24 ))
    BURN=640 FUSE=$f LAUNCHES=$L run fix6_f$f 200 python tools/time_fused.py
  done
  run benchdrv6 300 python bench.py --steps 20 --warmup 5
  PART=4 bash tools/r05_session.sh
  ;;
7)
  # refill rollouts (c4) and the info tap in fused launches: their tests; the landing_burn binary32
  # diagnostic; c4 at the whole swarm with refill against the one-launch-per-check rollout; the
  # two-level index's traffic (PMC)
  run gpu_t7 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "compaction or info_tap or launcher" -s
  run diag_lb 200 python tools/diag_f32_lb.py
  run c4_262k_refill 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0
  run c4_32k 300 python bench.py --workload c4 --steps 8 --warmup 2 --cpu-baseline 0
  V=psso-sac-for-powered-descent_amd/pdenv/libpdenv_idx2.so
  CASES="d_idx2:1:0:$V c_idx2:0:0:$V c_fine:0:0" run pmc7 900 bash tools/pmc_r05.sh
  ;;
8)
  # refill in batches (the first refill handed one particle per ended env, one atomic per wave
  # and step on the swarm's one counter: 12.5 ms a generation at 262 144 particles against 6.4 ms
  # without): the tests (incl. the binary32 teacher-forced bound by the step's conditioning), then
  # c4 at the whole swarm per batch size and off, c4 at 32 768 with refill forced on
  run gpu_t8 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "compaction or info_tap or launcher or f32_teacher" -s
  for b in 0 1 4 8 16 32; do
    run c4_262k_rf$b 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0 --policy-refill $b
  done
  for b in 0 8; do
    run c4_32k_rf$b 300 python bench.py --workload c4 --steps 8 --warmup 2 --cpu-baseline 0 --policy-refill $b
  done
  ;;
9)
  run gpu_t9 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "compaction or info_tap or launcher or f32_teacher" -s
  run c4_262k_auto 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0
  for b in 12 24; do
    run c4_262k_rf$b 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0 --policy-refill $b
  done
  ;;
10)
  run gpu_tests 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -s
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  run mlp_clocks 120 tools/bin/mlp_clocks
  run c4_262k_b24 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0
  run c4_262k_b0 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0 --policy-refill 0
  run benchdrv10 300 python bench.py --steps 20 --warmup 5
  ;;
11)
  for b in mlp_clocks mlp_clocks_v2 mlp_clocks_v2_kd2 mlp_clocks_v2_kd8 mlp_clocks_v2_kd16 mlp_clocks_v2_nt2kd8 \
           mlp_clocks_v2_noload mlp_clocks; do
    run clk_$b 60 tools/bin/$b
  done
  ;;
12)
  for b in mlp_clocks_v1 mlp_clocks_v3 mlp_clocks_v1_twice mlp_clocks_v2_twice mlp_clocks_v3_twice; do
    run clk12_$b 60 tools/bin/$b
  done
  run gpu_sac 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "sac or actor or c5" -s
  run c5_12 300 python bench.py --workload c5
  run c5_breakdown12 300 python tools/c5_breakdown.py
  ;;
13)
  for b in mlp_clocks_v3 mlp_clocks_v4 mlp_clocks_v4_twice; do
    run clk13_$b 60 tools/bin/$b
  done
  ;;
14)
  for n in 4096 2048 1024 512 128; do run clk14_v4_n$n 60 tools/bin/mlp_clocks_v4 $n; done
  for b in mlp_clocks_v4_nt2 mlp_clocks_v4_kd1 mlp_clocks_v4_kd3 mlp_clocks_v4_nt1kd4; do run clk14_$b 60 tools/bin/$b; done
  ;;
15)
  for b in mlp_clocks_v4 mlp_clocks_v5 mlp_clocks_v5; do run clk15_$b 60 tools/bin/$b; done
  ;;
16)
  for b in mlp_clocks_v5_loadonly mlp_clocks_v5_indep mlp_clocks_v6 mlp_clocks_v2_noload; do run clk16_$b 60 tools/bin/$b; done
  ;;
17)
  for b in mlp_clocks_v5_loadonly mlp_clocks_v5_loadonly_contig; do run clk17_$b 60 tools/bin/$b; done
  ;;
18)
  for b in mlp_clocks_v5 mlp_clocks_v7 mlp_clocks_v5 mlp_clocks_v7; do run clk18_$b 60 tools/bin/$b; done
  ;;
19)
  for b in n2r2 n2r3 n2r4 n4r2 n4r3 n1r4 n2r4; do run clk19_v7_$b 60 tools/bin/mlp_clocks_v7_$b; done
  ;;
20)
  for b in v7_n2r2 v8_n2r3 v8_n4r3 v8_n2r4 v8_n2r3; do run clk20_$b 60 tools/bin/mlp_clocks_$b; done
  ;;
21)
  for b in v8_nodma v8_nowread v8_nodma_nowread v8_n2r3; do run clk21_$b 60 tools/bin/mlp_clocks_$b; done
  ;;
22)
  for b in v7_n2r2 v9_n2 v9_n4 v9_n2; do run clk22_$b 60 tools/bin/mlp_clocks_$b; done
  ;;
23)
  run gpu_sac23 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "sac or actor or c5" -s
  run clk23_product 60 tools/bin/mlp_clocks
  run c5_23 300 python bench.py --workload c5
  run c5_breakdown23 300 python tools/c5_breakdown.py
  ;;
24)
  run gpu_sac24 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "sac or actor or c5 or fused" -s
  run c5_24 300 python bench.py --workload c5
  run c5_breakdown24 300 python tools/c5_breakdown.py
  BURN=640 FUSE=1 LAUNCHES=24 run fix24_f1 200 python tools/time_fused.py
  ;;
25)
  run gpu_t25 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "compaction or launcher" -s
  for c in "-1 -1" "0 24" "50 24" "90 24" "100 24" "75 8" "90 8" "90 16"; do
    set -- $c
    run c4_262k_own$1_b$2 300 python bench.py --workload c4 --particles 262144 --steps 6 --warmup 2 --cpu-baseline 0 \
        --policy-refill-own $1 --policy-refill $2
  done
  ;;
26)
  run gpu_tests 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  run bench 300 python bench.py
  run benchdrv 200 python bench.py --steps 20 --warmup 5
  run c4 200 python bench.py --workload c4
  run c4_262k 300 python bench.py --workload c4 --particles 262144 --steps 8 --warmup 2
  run c5 200 python bench.py --workload c5
  run c2 200 python bench.py --workload c2 --cpu-baseline 0
  ;;
27)
  STAGES="prof profdrv profc4 profc5" run profs 800 bash tools/gpu_session.sh
  run pmc 500 bash tools/pmc_r03b.sh
  ;;
28)
  P=psso-sac-for-powered-descent_amd/pdenv
  for r in 1 2; do
    for v in base smem sitilp silp sbias0; do
      lib=$P/libpdenv.so; [ $v != base ] && lib=$P/libpdenv_$v.so
      for d in 0 1; do
        PDENV_LIB=$lib DESCENT=$d BURN=640 FUSE=128 LAUNCHES=6 run t28_r${r}_${v}_d$d 200 python tools/time_fused.py
      done
    done
  done
  ;;
29)
  run gpu_t29 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "compaction or launcher" -s
  for r in 1 2; do
    for o in 1 0; do
      run c4_262k_order${o}_r$r 300 python bench.py --workload c4 --particles 262144 --steps 8 --warmup 3 --cpu-baseline 0 --policy-order $o
    done
  done
  PART=28 bash tools/r05_session.sh
  ;;
30)
  V=psso-sac-for-powered-descent_amd/pdenv/libpdenv_stamp0.so
  for f in 1 128; do
    L=$(( f > 1 ? 6 : 40 ))
    PDENV_LIB=$V N=4096 LPE=16 WIND=0 TILT=0 STATS=1 FUSE=$f LAUNCHES=$L BURN=256 run st30_f$f 200 python tools/time_fused.py
    N=4096 LPE=16 WIND=0 TILT=0 FUSE=$f LAUNCHES=$L BURN=256 run t30_f$f 200 python tools/time_fused.py
  done
  ;;
31)
  PART=28 bash tools/r05_session.sh && PART=30 bash tools/r05_session.sh
  ;;
32)
  run gpu_c3_32 900 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
      --timeout-method thread -k "c3 or fused or ragged or teacher"
  for r in 1 2; do for d in 0 1; do
    DESCENT=$d BURN=640 FUSE=128 LAUNCHES=6 run t32_r${r}_d$d 200 python tools/time_fused.py
  done; done
  run benchdrv32 200 python bench.py --steps 20 --warmup 5
  ;;
33)
  PART=26 bash tools/r05_session.sh
  ;;
34)
  PART=27 bash tools/r05_session.sh
  ;;
35)
  P=psso-sac-for-powered-descent_amd/pdenv
  for r in 1 2; do
    for v in base mc32 mctrk mcnorp ilptrk; do
      lib=$P/libpdenv.so; [ $v != base ] && lib=$P/libpdenv_$v.so
      for d in 0 1; do
        PDENV_LIB=$lib DESCENT=$d BURN=640 FUSE=128 LAUNCHES=6 run t35_r${r}_${v}_d$d 200 python tools/time_fused.py
      done
    done
  done
  ;;
36)
  for r in 1 2; do
    for b in 0 24; do
      run c4_32k_36_rf${b}_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0 --policy-refill $b
    done
  done
  ;;
37)
  run clk37_v10 60 tools/bin/mlp_clocks_v10
  run gpu_sac37 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "sac or actor or c5 or fused" -s
  run c5_37 300 python bench.py --workload c5
  run c5_breakdown37 300 python tools/c5_breakdown.py
  ;;
38)
  run gpu_pol38 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "policy or pso or compaction or c4 or drivers or swarm" -s
  run c4_38 300 python bench.py --workload c4
  run c4_262k_38 300 python bench.py --workload c4 --particles 262144 --steps 8 --warmup 2 --cpu-baseline 0
  ;;
39)
  PART=26 bash tools/r05_session.sh
  ;;
40)
  PART=27 bash tools/r05_session.sh
  ;;
50)
  PART=26 bash tools/r05_session.sh
  ;;
41)
  A="--steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 --descent 0 --fresh 0 --others 0"
  for r in 1 2 3; do
    run sp41_base_$r 200 python tools/spin_probe.py --spin 0 -- $A
    run sp41_spin_$r 200 python tools/spin_probe.py --spin 1 -- $A
    HIP_FORCE_DEV_KERNARG=1 run sp41_karg_$r 200 python tools/spin_probe.py --spin 0 -- $A
    HIP_FORCE_DEV_KERNARG=1 run sp41_both_$r 200 python tools/spin_probe.py --spin 1 -- $A
  done
  ;;
42)
  for r in 1 2 3; do
    run c5g1_$r 200 python bench.py --workload c5 --cpu-baseline 0 --graph 1
    run c5g0_$r 200 python bench.py --workload c5 --cpu-baseline 0 --graph 0
  done
  for g in 1 0; do
    run c5trace_g$g 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5trace_g$g -o run -- python3 bench.py --workload c5 --cpu-baseline 0 --steps 192 --warmup 32 --graph $g
  done
  ;;
43)
  run gpu_sac43 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "sac or actor or c5 or collector" -s
  run c5_43a 300 python bench.py --workload c5
  run c5_43b 300 python bench.py --workload c5
  run bench43 600 python bench.py
  ;;
44)
  run c5_44a 300 python bench.py --workload c5
  run c5_44b 300 python bench.py --workload c5
  run c5prof44 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof44 -o run -- python3 bench.py --workload c5
  ;;
45)
  run gpu_pso45 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "policy or pso or compaction or c4 or drivers or swarm or migrat or share" -s
  run c4_45a 300 python bench.py --workload c4
  run c4_45b 300 python bench.py --workload c4
  STAGES="profc4" run profs45 800 bash tools/gpu_session.sh
  ;;
46|47|48|49|51)
  PART=45 bash tools/r05_session.sh
  ;;
esac
echo "=== done"
