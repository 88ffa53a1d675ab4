#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.  Every GPU step has its
# own time limit; a crash/timeout/abort stops the session (no further GPU work).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stage() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STAGES=${STAGES:-"tests smoke bench prof"}
for s in $STAGES; do
  case $s in
    draws) stage gpu_draws 600 python -u -m pytest tests/test_gpu_draws.py tests/test_gpu_c3.py -x -v --timeout 300 --timeout-method thread ;;
    tests) stage gpu_tests 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread ;;
    testsall) stage gpu_tests 900 python -u -m pytest tests/ -m gpu -q --timeout 120 --timeout-method thread ;;
    smoke) stage smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) stage bench 600 python bench.py ;;
    benchdrv) stage benchdrv 600 python bench.py --steps 20 --warmup 5 ;;
    bench32) stage bench32 600 python bench.py --precision f32 ;;
    c2) stage c2 600 python bench.py --workload c2 --cpu-baseline 0 ;;
    c2rk4) stage c2rk4 600 python bench.py --workload c2 --integrator rk4 --cpu-baseline 0 ;;
    prof) stage prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 192 --warmup 32 --cpu-baseline 0 --secondary 0 --others 0 --descent 1 ;;
    profc4) stage profc4 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc4 -o run -- python3 bench.py --workload c4 --steps 16 --warmup 2 --cpu-baseline 0 ;;
    profc5) stage profc5 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc5 -o run -- python3 bench.py --workload c5 --steps 192 --warmup 32 ;;
    profdrv) stage profdrv 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profdrv -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --secondary 0 --others 0 --descent 1 ;;
    prof32) stage prof32 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof32 -o run -- python3 bench.py --steps 96 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0 --precision f32 ;;
    sweep) stage sweep 600 python tools/sweep.py ;;
    plpe) stage plpe 600 python tools/policy_lpe_sweep.py ;;
    c4) stage c4 600 python bench.py --workload c4 ;;
    c5) stage c5 600 python bench.py --workload c5 ;;
    c3d) stage c3d 600 python bench.py --workload c3-descent --secondary 0 --cpu-baseline 0 ;;
    pmc) stage pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0
         stage pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0 ;;
    pmc32) stage pmc_fetch32 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch32 -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0 --precision f32
         stage pmc_write32 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write32 -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0 --precision f32 ;;
    pmcmix) stage pmc_mix 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_mix -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0
         stage pmc_mix2 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mix2 -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0 ;;
    avail) stage avail 300 rocprofv3 --list-avail ;;
    pmcv) stage pmc_valu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_valu -o run -- python3 bench.py --steps 32 --warmup 16 --cpu-baseline 0 --secondary 0 --others 0 ;;
  esac
done
echo "=== done"
