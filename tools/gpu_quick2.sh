#!/bin/bash
# quick check of the committed kernel: GPU tests, bench (config 2 + extras, no CPU leg), clock
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-q}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err && cat gpurun_out/bench_$T.json \
 && RHP_LIB=$PWD/libreactorng_amd/librhp_clock.so timeout -k 10 200 python tools/kclock.py 2>&1 | grep -v amdgpu.ids
