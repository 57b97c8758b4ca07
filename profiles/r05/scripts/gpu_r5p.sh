#!/bin/bash
# round 5 session p: chunked -- the body's edge blocks stored as whole lines (RHP_WHOLE_EDGES) instead of byte by byte
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5p && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
RHP_LIB=$L/librhp_x_we.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "chunk or golden or fuzz" > gpurun_out/r5p/pytest_we.log 2>&1 && tail -2 gpurun_out/r5p/pytest_we.log || exit 1
for r in 1 2; do
  for v in cur we; do
    RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config chunked --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5p/chunked_$v.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r5p/chunked_$v.json')); print('$v', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5p/ab.txt
  done
done
echo SESSION_OK
