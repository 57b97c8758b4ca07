#!/bin/bash
# round 5 session aa: the burst test's GPU/host ratio over three runs (the guard's margin)
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5aa && export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread -m gpu tests/test_reactor.py -k burst_rounds_gpu_vs_host > gpurun_out/r5aa/burst_$r.log 2>&1 || { grep -h "burst req/s\|assert" gpurun_out/r5aa/burst_$r.log; exit 1; }
  grep -h "burst req/s" gpurun_out/r5aa/burst_$r.log
done
echo SESSION_OK
