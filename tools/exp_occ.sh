#!/bin/bash
# occupancy / structure experiments on config 2: "lib:waves" pairs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-occ}
for lw in ${LIBS_WAVES}; do
  l=${lw%%:*}; w=${lw##*:}
  RHP_LIB=$PWD/libreactorng_amd/$l.so RHP_WAVES=$w timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 5 --config ${CFG:-get256} > gpurun_out/${TAG}_${l}_w$w.json 2>gpurun_out/${TAG}_${l}_w$w.err || exit 1
  echo "$l waves=$w $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${l}_w$w.json'));print(d['value'],d['roofline']['kernel_ms'],d['config']['ok_fraction'])")"
done
