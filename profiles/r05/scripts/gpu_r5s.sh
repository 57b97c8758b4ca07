#!/bin/bash
# round 5 session s: stamps of the committed kernel for config 5 (compact records) and chunked
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5s && export TMPDIR=/tmp
RHP_LIB=$PWD/libreactorng_amd/librhp_x_stamps.so STAMPS_CFG=6 timeout -k 10 300 python tools/stamps2.py > gpurun_out/r5s/stamps_c5_chunked.txt 2>&1 && head -60 gpurun_out/r5s/stamps_c5_chunked.txt && echo SESSION_OK
