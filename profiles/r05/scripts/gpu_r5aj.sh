#!/bin/bash
# round 5 session aj: config 3 workgroup ends against their ranges' work
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5aj && export TMPDIR=/tmp
RHP_LIB=$PWD/libreactorng_amd/librhp_x_stamps.so timeout -k 10 300 python tools/stamps_wg.py > gpurun_out/r5aj/stamps_wg.txt 2>&1 && cat gpurun_out/r5aj/stamps_wg.txt && echo SESSION_OK
