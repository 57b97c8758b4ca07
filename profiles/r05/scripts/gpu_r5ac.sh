#!/bin/bash
# round 5 session ac: an uneven range's order in one wave's staging when it fits (15 walking waves, ow) against two
# (14, cur); parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5ac && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
RHP_LIB=$L/librhp_x_ow.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_line_windows.py > gpurun_out/r5ac/pytest_ow.log 2>&1 && tail -2 gpurun_out/r5ac/pytest_ow.log || exit 1
for r in 1 2 3; do
  for v in cur ow; do
    RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config zipf --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5ac/zipf_$v.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r5ac/zipf_$v.json')); print('$v', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5ac/ab.txt
  done
done
echo SESSION_OK
