cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk4.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rk4_tests.log 2>&1; rc=$?; tail -12 gpurun_out/rk4_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c2 --integrator rk4 --secondary 0 > gpurun_out/bench_c2_rk4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2_rk4.log
timeout -k 10 300 python bench.py --workload c2 --secondary 0 > gpurun_out/bench_c2_ref.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2_ref.log
