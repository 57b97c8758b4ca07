mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_framing.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_wexit.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_wexit.log; [ $rc -eq 0 ] || exit $rc
LIBS="base wexit" ROUNDS=3 TAG=wexit bash tools/gpu_ab2.sh
