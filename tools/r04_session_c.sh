#!/bin/bash
# Round-4 session C, in parts (PART=1|2|3), each under its own gpurun call:
#   1: the round-4 kernel changes timed against variants built without each (c3 and c3-descent,
#      128 steps per launch, two interleaved rounds): nowqx = no workgroup query exchange
#      (-DPD_WQX=0), nomk = IEEE divisions for the known divisors (-DPD_MARKSTEIN=0), noat = the
#      device library's atan2 (-DPD_ATAN2_FD=0); then c2 (4 096 envs, no wind) at LPE 16 / 8 / 2.
#   2: the bench lines (driver command, defaults, c4, c5), the policy lanes-per-env sweep, and
#      rocprofv3 kernel traces of the default, driver-command, c4 and c5 runs.
#   3: PMC passes (tools/pmc_r03b.sh: traffic, instruction mix, waits and LDS, c3 and c3-descent).
# Variants: python -c "from pdenv import build as b; b.build_variant('nowqx', ['-DPD_WQX=0'])" etc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
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
  for d in 1 0; do
    VARIANTS="base nowqx nomk noat" FUSE=128 LAUNCHES=6 DESCENT=$d run exp_r04_d$d 500 bash tools/exp_session.sh
  done
  for l in 16 8 2; do
    N=4096 WIND=0 TILT=0 LPE=$l FUSE=128 LAUNCHES=6 run c2_lpe$l 200 python tools/time_fused.py
  done ;;
2)
  run benchdrv 400 python bench.py --steps 20 --warmup 5
  run bench 400 python bench.py
  run c4 300 python bench.py --workload c4
  run c5 300 python bench.py --workload c5
  run plpe 300 python tools/policy_lpe_sweep.py
  STAGES="prof profdrv profc4 profc5" run profs 900 bash tools/gpu_session.sh ;;
3)
  run pmc 900 bash tools/pmc_r03b.sh ;;
4)
  # after part 1 (the exchange 20-25 % slower, atan2_fd slower than the library's): base = no
  # exchange; at0 = library atan2, mk0 = IEEE divisions, wqx1 = the exchange; c2 (4 096 envs, no
  # wind): pieces at LPE 16 / 8 (base) against payload sums (c2pl0) and the library atan2 (c2at0)
  run gpu_lpe_tests 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "batched_random or ragged or step_n_fused or sac or device_solve or cell_pieces"
  for d in 1 0; do
    VARIANTS="base at0 mk0 wqx1" FUSE=128 LAUNCHES=6 DESCENT=$d run exp_r04b_d$d 500 bash tools/exp_session.sh
  done
  for l in 16 8; do
    VARIANTS="base c2pl0 c2at0" N=4096 WIND=0 TILT=0 LPE=$l FUSE=128 LAUNCHES=6 run exp_r04b_c2_lpe$l 300 bash tools/exp_session.sh
  done ;;
5)
  # the build with the measured defaults (no exchange, library atan2, pieces at LPE 4/8): the GPU
  # suite and smoke, c3 / c3-descent at LPE 1 and 2, the bench lines
  run gpu_tests 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for d in 0 1; do for l in 2 1; do
    LPE=$l FUSE=128 LAUNCHES=6 DESCENT=$d run lpe_c3_d${d}_l$l 200 python tools/time_fused.py
  done; done
  run benchdrv 300 python bench.py --steps 20 --warmup 5
  run bench 400 python bench.py ;;
6)
  run c4 300 python bench.py --workload c4
  run c5 300 python bench.py --workload c5
  run c2 300 python bench.py --workload c2 --cpu-baseline 0
  run plpe 300 python tools/policy_lpe_sweep.py
  STAGES="prof profdrv profc4 profc5" run profs 700 bash tools/gpu_session.sh ;;
7)
  # PD_STAMP section clocks of the c3 kernel (libpdenv_stamp.so: build_variant('stamp',
  # ['-DPD_STAMP'])), then the PMC passes (traffic, instruction mix, waits / LDS)
  for d in 0 1; do
    STATS=1 DESCENT=$d FUSE=128 LAUNCHES=3 PDENV_LIB=psso-sac-for-powered-descent_amd/pdenv/libpdenv_stamp.so \
      run stamp_d$d 200 python tools/time_fused.py
  done
  run pmc 900 bash tools/pmc_r03b.sh ;;
8)
  # c5 in one launch (pd_step_sac_fused): its tests, the c5 line and its rocprofv3 trace
  run gpu_sac_tests 400 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "sac"
  run c5 300 python bench.py --workload c5
  STAGES="profc5" run profs 300 bash tools/gpu_session.sh ;;
9)
  # after the fault of part 8 (the SAC launcher dispatched the non-SAC kernel for pd_step_sac_fused:
  # a NULL action pointer): the suite, smoke, the tabulated atmosphere / inertia timed against
  # their exact formulas (PDENV_ATM_TAB=0), c5, c2 and the bench line
  run gpu_tests 700 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for r in 1 2; do for d in 0 1; do
    FUSE=128 LAUNCHES=6 DESCENT=$d run atm_d${d}_r$r 200 python tools/time_fused.py
    PDENV_ATM_TAB=0 FUSE=128 LAUNCHES=6 DESCENT=$d run atm0_d${d}_r$r 200 python tools/time_fused.py
  done; done
  run c5 300 python bench.py --workload c5
  run c2 300 python bench.py --workload c2 --cpu-baseline 0
  run bench 400 python bench.py ;;
10)
  # part 9: the tables made c3 / c3-descent slower (0.0330 / 0.0391 against 0.0315 / 0.0363) and
  # c2, c4, c5, f32 faster: which table, and the code-size effect (notab: built without them)
  L=psso-sac-for-powered-descent_amd/pdenv
  for r in 1 2; do for d in 0 1; do
    FUSE=128 LAUNCHES=6 DESCENT=$d run tab_both_d${d}_r$r 200 python tools/time_fused.py
    PDENV_ATM_ONLY=inr FUSE=128 LAUNCHES=6 DESCENT=$d run tab_inr_d${d}_r$r 200 python tools/time_fused.py
    PDENV_ATM_ONLY=atm FUSE=128 LAUNCHES=6 DESCENT=$d run tab_atm_d${d}_r$r 200 python tools/time_fused.py
    PDENV_ATM_TAB=0 FUSE=128 LAUNCHES=6 DESCENT=$d run tab_none_d${d}_r$r 200 python tools/time_fused.py
    PDENV_LIB=$L/libpdenv_notab.so FUSE=128 LAUNCHES=6 DESCENT=$d run tab_notab_d${d}_r$r 200 python tools/time_fused.py
    # ro: each sub-step's end atmosphere computed before atan2 (its loads overlap atan2's work)
    PDENV_LIB=$L/libpdenv_ro.so FUSE=128 LAUNCHES=6 DESCENT=$d run tab_ro_d${d}_r$r 200 python tools/time_fused.py
    PDENV_LIB=$L/libpdenv_ro.so PDENV_ATM_ONLY=inr FUSE=128 LAUNCHES=6 DESCENT=$d run tab_roinr_d${d}_r$r 200 python tools/time_fused.py
    PDENV_LIB=$L/libpdenv_ronotab.so FUSE=128 LAUNCHES=6 DESCENT=$d run tab_ronotab_d${d}_r$r 200 python tools/time_fused.py
  done; done
  for r in 1 2; do
    N=4096 WIND=0 TILT=0 FUSE=128 LAUNCHES=6 run tab_c2_both_r$r 200 python tools/time_fused.py
    PDENV_ATM_ONLY=inr N=4096 WIND=0 TILT=0 FUSE=128 LAUNCHES=6 run tab_c2_inr_r$r 200 python tools/time_fused.py
    PDENV_LIB=$L/libpdenv_c2notab.so N=4096 WIND=0 TILT=0 FUSE=128 LAUNCHES=6 run tab_c2_notab_r$r 200 python tools/time_fused.py
    PREC=f32 FUSE=128 LAUNCHES=6 run tab_f32_both_r$r 200 python tools/time_fused.py
    PREC=f32 PDENV_ATM_ONLY=inr FUSE=128 LAUNCHES=6 run tab_f32_inr_r$r 200 python tools/time_fused.py
    PREC=f32 PDENV_LIB=$L/libpdenv_f32notab.so FUSE=128 LAUNCHES=6 run tab_f32_notab_r$r 200 python tools/time_fused.py
  done ;;
11)
  # the build after part 10 (no inertia table; the atmosphere table for binary32 and the windless
  # kernels only): the suite, smoke, the kernels timed, c4 with the live list switched on mid-rollout
  # (PDENV_COMPACT_AT) or from the start (PDENV_COMPACT=1), c5, the bench line
  run gpu_tests 700 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for d in 0 1; do FUSE=128 LAUNCHES=6 DESCENT=$d run k_d$d 200 python tools/time_fused.py; done
  PREC=f32 FUSE=128 LAUNCHES=6 run k_f32 200 python tools/time_fused.py
  N=4096 WIND=0 TILT=0 FUSE=128 LAUNCHES=6 run k_c2 200 python tools/time_fused.py
  run c4 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  PDENV_COMPACT_AT=0.5 run c4_at50 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  PDENV_COMPACT_AT=0.2 run c4_at20 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  PDENV_COMPACT=1 run c4_list 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  run c5 300 python bench.py --workload c5
  run bench 400 python bench.py ;;
12)
  # the final build's measurement: the suite, smoke, the bench lines (defaults and the driver's
  # command), c4 / c5 / c2, rocprofv3 kernel traces (default, driver command, c4, c5) and the PMC
  # passes (c3, c3-descent); tools/collect_r03.py r04 reduces them into profiles/
  run gpu_tests 700 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  run bench 400 python bench.py
  run benchdrv 300 python bench.py --steps 20 --warmup 5
  run c4 300 python bench.py --workload c4
  # (the list launches with the parameter copy, switched on at 50 / 25 % live: PDENV_COMPACT_AT)
  PDENV_COMPACT_AT=0.5 run c4_at50 300 python bench.py --workload c4 --cpu-baseline 0
  PDENV_COMPACT_AT=0.25 run c4_at25 300 python bench.py --workload c4 --cpu-baseline 0
  run c5 300 python bench.py --workload c5
  run c2 300 python bench.py --workload c2 --cpu-baseline 0
  STAGES="prof profdrv profc4 profc5" run profs 600 bash tools/gpu_session.sh
  run pmc 600 bash tools/pmc_r03b.sh ;;
13)
  # c4's list launches with the live envs' actor parameters copied once per launch (libpdenv_pwc:
  # build_variant('pwc', [], unit=(0, 1, 0), host=True)): the compaction invariance test on it, then
  # c4 with the list off / switched on at 50 % and 25 % live / on from the start
  L=psso-sac-for-powered-descent_amd/pdenv/libpdenv_pwc.so
  PDENV_LIB=$L run pwc_tests 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "compaction_invariant or policy_rollout or pso_driver"
  for r in 1 2; do
    PDENV_LIB=$L run pwc_c4_off_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_LIB=$L PDENV_COMPACT_AT=0.5 run pwc_c4_at50_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_LIB=$L PDENV_COMPACT_AT=0.25 run pwc_c4_at25_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_LIB=$L PDENV_COMPACT=1 run pwc_c4_list_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  done ;;
14)
  # the actor split over the env's lane pair (PD_ACTOR_SPLIT; libpdenv_nosplit: build_variant(
  # 'nosplit', ['-DPD_ACTOR_SPLIT=0'], unit=(0, 1, 0)) has the landing-burn kernels without it):
  # the policy tests, c4 with and without it (two rounds), the policy lanes-per-env sweep, a c4
  # kernel trace (both libraries were built with the four-parameters-per-thread k_pso_step, reverted after)
  L=psso-sac-for-powered-descent_amd/pdenv/libpdenv_nosplit.so
  run split_tests 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "policy or pso or compaction or actor or drivers"
  for r in 1 2; do
    run split_c4_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_LIB=$L run nosplit_c4_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  done
  run plpe 300 python tools/policy_lpe_sweep.py
  STAGES="profc4" run profs 300 bash tools/gpu_session.sh ;;
15)
  # policy waves leave the launch once their episodes have all ended (PD_POL_EXIT; libpdenv_noexit:
  # build_variant('noexit', ['-DPD_POL_EXIT=0'], unit=(0, 1, 0))): the policy tests, then c4 with and
  # without it at 8 and 16 policy steps per launch (PDENV_PFUSE), two rounds
  L=psso-sac-for-powered-descent_amd/pdenv/libpdenv_noexit.so
  run exit_tests 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "policy or pso or compaction or actor or drivers"
  for r in 1 2; do
    run exit_c4_f8_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_LIB=$L run noexit_c4_f8_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_PFUSE=16 run exit_c4_f16_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_PFUSE=16 PDENV_LIB=$L run noexit_c4_f16_r$r 300 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  done ;;
16)
  # part 15 and the final measurement (part 12) in one call: the suite and smoke; c4 with and
  # without the policy waves' exit at 8 / 16 policy steps per launch; the bench lines, c4 / c5 / c2,
  # rocprofv3 kernel traces and the PMC passes of this build
  L=psso-sac-for-powered-descent_amd/pdenv/libpdenv_noexit.so
  run gpu_tests 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for r in 1 2; do
    run exit_c4_f8_r$r 200 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_LIB=$L run noexit_c4_f8_r$r 200 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
    PDENV_PFUSE=16 run exit_c4_f16_r$r 200 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  done
  run bench 300 python bench.py
  run benchdrv 200 python bench.py --steps 20 --warmup 5
  run c4 200 python bench.py --workload c4
  run c5 200 python bench.py --workload c5
  run c2 200 python bench.py --workload c2 --cpu-baseline 0
  STAGES="prof profdrv profc4 profc5" run profs 500 bash tools/gpu_session.sh
  run pmc 500 bash tools/pmc_r03b.sh ;;
17)
  # the default of 16 policy steps per launch (part 16: 8 -> 16 with the waves' exit, -5 %): the
  # policy tests on it, c4 at 16 / 32 / 64 steps per launch (two rounds), the c4 line and its trace
  run pf_tests 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "policy or pso or compaction or actor or drivers"
  for r in 1 2; do for f in 16 32 64; do
    PDENV_PFUSE=$f run pf${f}_c4_r$r 200 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0
  done; done
  run c4 200 python bench.py --workload c4
  STAGES="profc4" run profs 300 bash tools/gpu_session.sh ;;
18)
  # the final build (64 policy steps per launch, part 17): the suite and smoke, c4 (two rounds and
  # the line), its trace, the bench lines
  run gpu_tests 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  for r in 1 2; do run pf64_c4_r$r 200 python bench.py --workload c4 --steps 32 --warmup 4 --cpu-baseline 0; done
  run c4 200 python bench.py --workload c4
  run bench 300 python bench.py
  run benchdrv 200 python bench.py --steps 20 --warmup 5
  STAGES="profc4 prof profdrv" run profs 400 bash tools/gpu_session.sh ;;
19)
  # the committed tree as the round-end driver runs it: the GPU suite, smoke, the default bench line
  run gpu_tests 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
  run bench 300 python bench.py ;;
esac
echo "=== done"
