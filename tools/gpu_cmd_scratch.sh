mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_ceiling > gpurun_out/ceiling.txt 2>&1; cat gpurun_out/ceiling.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "last_len or 4gib" > gpurun_out/pytest_lastlen.log 2>&1; tail -3 gpurun_out/pytest_lastlen.log
LIBS="base prio8" ROUNDS=2 TAG=prio bash tools/gpu_ab2.sh
