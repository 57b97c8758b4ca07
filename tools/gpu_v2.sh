#!/bin/bash
# One GPU session for a kernel revision: parity tests, bench variants (waves per
# workgroup), rocprofv3 kernel-trace summary, DFA-step microbenchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-v2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
  && echo PYTEST_OK || { tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
for w in ${WAVES_LIST:-16}; do
  RHP_WAVES=$w timeout -k 10 180 python bench.py --no-cpu --steps 50 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench_${TAG}_w$w.json 2>gpurun_out/bench_${TAG}_w$w.err || { tail -5 gpurun_out/bench_${TAG}_w$w.err; exit 1; }
  echo "waves=$w $(python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_w$w.json'));print(d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['config']['ok_fraction'])")"
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG} -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 && echo PROF_OK || exit 1
fi
if [ -n "$UBENCH" ]; then
  timeout -k 10 120 ./tools/ubench_dfa2 > gpurun_out/ubench_${TAG}.txt 2>&1 && cat gpurun_out/ubench_${TAG}.txt
fi
