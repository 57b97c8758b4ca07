#!/bin/bash
# round 5 session c: H2D probe (the reactor round's copy), stamps with the early form's C-E split
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5c && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
timeout -k 10 120 tools/h2d_probe > gpurun_out/r5c/h2d_probe.txt 2>&1 && echo H2D_OK && cat gpurun_out/r5c/h2d_probe.txt \
 && RHP_LIB=$L/librhp_x_stampspl.so STAMPS_CFG=2,3 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5c/stamps_pl.txt 2>&1 && echo STAMPS_OK && head -12 gpurun_out/r5c/stamps_pl.txt
