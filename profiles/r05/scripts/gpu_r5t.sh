#!/bin/bash
# round 5 session t: the replay's rounds claimed from an LDS counter (faster waves take more) against rounds dealt
# out by wave index; parity first, stamps of chunked after
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5t && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
RHP_LIB=$L/librhp_x_dyn.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_sessions.py tests/test_line_windows.py > gpurun_out/r5t/pytest_dyn.log 2>&1 && tail -2 gpurun_out/r5t/pytest_dyn.log || exit 1
for r in 1 2; do
  for v in cur dyn; do
    for c in chunked post zipf; do
      RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5t/${c}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r5t/${c}_$v.json')); print('$v', '$c', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5t/ab.txt
    done
  done
done
RHP_LIB=$L/librhp_x_stamps.so STAMPS_CFG=6 timeout -k 10 300 python tools/stamps2.py > gpurun_out/r5t/stamps_chunked_dyn.txt 2>&1 && grep -A8 "exit" gpurun_out/r5t/stamps_chunked_dyn.txt | head -20 && echo SESSION_OK
