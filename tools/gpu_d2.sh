#!/bin/bash
# decode/walk A/B: parity on the default build, then bench base vs variants, stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-d2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 && echo PYTEST_OK || { tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
TAG=$TAG LIBS_WAVES="${LIBS_WAVES:-librhp_base:16 librhp:16 librhp_d32:16}" CFGS="${CFGS:-get256 zipf post}" bash tools/exp_cfg.sh && LIBS_CFG="${LIBS_CFG:-librhp_stamps:2 librhp_stamps:3}" bash tools/stamps_ab.sh
