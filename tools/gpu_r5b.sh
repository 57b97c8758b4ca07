#!/bin/bash
# round 5 session b: line-window diagnostic (time + FETCH of config 3), SQ counters per config on the
# new decode, reactor round timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5b && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
for v in dx ladiag; do
  RHP_LIB=$L/librhp_x_$v.so RHP_BENCH_DIAG=1 timeout -k 10 300 python bench.py --config zipf --extra none --no-cpu --no-e2e --steps 30 --warmup 5 \
    > gpurun_out/r5b/zipf_$v.json 2>/dev/null || exit 1
  RHP_LIB=$L/librhp_x_$v.so RHP_BENCH_DIAG=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5b/pmc_${v}_zipf -o p \
    -- python3 bench.py --config zipf --extra none --steps 6 --warmup 2 --no-cpu --no-e2e > gpurun_out/r5b/pmc_${v}_zipf.log 2>&1 || exit 1
done && echo LADIAG_OK \
 && for c in get256 zipf post chunked; do TAG=r5b/sq_$c CONFIG=$c RHP_LIB=$L/librhp_x_dx.so bash tools/pmc_sq.sh > gpurun_out/r5b/sq_$c.txt 2>&1 || exit 1; done && echo SQ_OK \
 && timeout -k 10 600 bash tools/reactor_timeline.sh > gpurun_out/r5b/reactor_timeline.txt 2>&1 && echo TIMELINE_OK
