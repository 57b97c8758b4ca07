#!/bin/bash
# timing experiment: pool chunk size (RHP_CHUNK) for each config
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-chunk}
for cfg in ${CONFIGS:-get256}; do for c in ${CHUNKS:-256 128 64}; do
RHP_CHUNK=$c timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 --config $cfg > gpurun_out/${TAG}_${cfg}_c$c.json 2>/dev/null || exit 1
echo "$cfg chunk=$c $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${cfg}_c$c.json'));print(d['value'],d['roofline']['kernel_ms'])")"
done; done
