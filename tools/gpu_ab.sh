#!/bin/bash
# parity tests on the in-tree kernel, then bench it against alternative builds (RHP_LIB)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-ab}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_${TAG}.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
fi
for cfg in ${CONFIGS:-get256}; do
for l in libreactorng_amd/librhp.so ${ALT_LIBS}; do
  b=$(basename $l .so)
  RHP_LIB=$PWD/$l timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 5 --config $cfg ${BENCH_ARGS} > gpurun_out/${TAG}_${cfg}_$b.json 2>gpurun_out/${TAG}_${cfg}_$b.err || exit 1
  echo "$cfg $b $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${cfg}_$b.json'));print(d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'])")"
done
done
