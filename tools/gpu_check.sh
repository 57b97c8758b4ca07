#!/bin/bash
# One GPU session: parity tests, bench line, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with && so a failure
# or fault stops the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu_${TAG}.log 2>&1 \
 && echo "pytest gpu OK" \
 && timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && cat gpurun_out/bench_${TAG}.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG} -o run \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 \
 && echo "rocprof OK"
