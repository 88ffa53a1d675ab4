cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -x -k "teacher or batched or config1" > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/gpu_tests.log
LPES=1,2,4 timeout -k 10 300 python tools/sweep.py > gpurun_out/sweep.log 2>&1; echo "sweep rc=$?"
