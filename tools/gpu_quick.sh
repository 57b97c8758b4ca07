#!/bin/bash
# parity tests + bench variants (RHP_WAVES) in one call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-quick}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_${TAG}.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
for w in ${WAVES_LIST:-16}; do
  RHP_WAVES=$w timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG}_w$w.json 2>gpurun_out/${TAG}_w$w.err || exit 1
  echo "waves=$w $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_w$w.json'));print(d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'])")"
done
