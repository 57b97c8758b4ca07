#!/bin/bash
# Round-end evidence for the committed kernel: full GPU test suite, the bench
# line (with the CPU baseline), rocprofv3 kernel-trace summary of the same
# workload, PMC passes (HBM traffic), end-to-end PCIe rate.  Every GPU step has
# its own time limit; steps are chained with && so a failure stops the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-final}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
 && echo PYTEST_OK \
 && timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
 && cat gpurun_out/bench_${TAG}.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG} -o run \
      -- python3 bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/prof_${TAG}.log 2>&1 \
 && echo PROF_OK \
 && TAG=pmc_${TAG} bash tools/pmc_probe.sh \
 && timeout -k 10 300 python tools/e2e_pcie.py > gpurun_out/e2e_${TAG}.json 2> gpurun_out/e2e_${TAG}.err \
 && cat gpurun_out/e2e_${TAG}.json
