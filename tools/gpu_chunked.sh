#!/bin/bash
# Chunked-body path on the GPU: its parity tests, then the chunked config timed
# with this library and (if present) with an older one (RHP_OLD, e.g. a build of
# the previous commit) at a smaller size.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-ck}
OLD=${RHP_OLD:-libreactorng_amd/librhp_x_old.so}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/pytest_$T.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_$T.log
[ $rc -eq 0 ] || exit $rc
for n in 262144 1048576; do
  timeout -k 10 300 python -u bench.py --config chunked --extra none --no-cpu --no-e2e --steps 10 --warmup 2 --per-gpu $n \
    > gpurun_out/bench_${T}_new_$n.json 2> gpurun_out/bench_${T}_new_$n.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('new', sys.argv[2], d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms', d['config']['ok_fraction'])" gpurun_out/bench_${T}_new_$n.json $n
done
if [ -f "$OLD" ]; then
  RHP_LIB=$PWD/$OLD timeout -k 10 400 python -u bench.py --config chunked --extra none --no-cpu --no-e2e --steps 3 --warmup 1 \
    --per-gpu 65536 > gpurun_out/bench_${T}_old.json 2> gpurun_out/bench_${T}_old.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('old 65536', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms', d['config']['ok_fraction'])" gpurun_out/bench_${T}_old.json
  timeout -k 10 300 python -u bench.py --config chunked --extra none --no-cpu --no-e2e --steps 3 --warmup 1 --per-gpu 65536 \
    > gpurun_out/bench_${T}_new_65536.json 2>> gpurun_out/bench_${T}_new.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('new 65536', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')" gpurun_out/bench_${T}_new_65536.json
fi
echo CHUNKED_OK
