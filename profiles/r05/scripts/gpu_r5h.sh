#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5h && export TMPDIR=/tmp
timeout -k 10 120 tools/h2d_probe 2>&1 | head -6 | tee gpurun_out/r5h/h2d_cpu.txt
