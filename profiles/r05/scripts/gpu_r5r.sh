#!/bin/bash
# round 5 session r: a 1M-request GPU fuzz against the oracle (every layout, phr and http, max_headers 0-64) and
# config 2's kernel time / traffic against batch size for the committed kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5r && export TMPDIR=/tmp
timeout -k 10 900 python -u tools/fuzz_gpu_big.py 1048576 1 > gpurun_out/r5r/fuzz_gpu_big.txt 2>&1 && tail -2 gpurun_out/r5r/fuzz_gpu_big.txt \
 && TAG=r5 timeout -k 10 900 bash tools/gpu_size_scaling.sh && cat gpurun_out/size_scaling_r5.txt && echo SESSION_OK
