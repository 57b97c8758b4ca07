#!/bin/bash
# timing experiments: RHP_EXPERIMENT bits (1 = cache-resident windows, 2 = no record stores) x RHP_WAVES
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-exp}
for x in ${XS:-0 1 2 3}; do for w in ${WS:-16}; do
RHP_EXPERIMENT=$x RHP_WAVES=$w timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}_x${x}_w$w.json 2>/dev/null || exit 1
echo "exp=$x waves=$w $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_x${x}_w$w.json'));print(d['value'],d['roofline']['kernel_ms'])")"
done; done
