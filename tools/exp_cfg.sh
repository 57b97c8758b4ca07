#!/bin/bash
# bench several libs x configs: LIBS_WAVES="lib:waves ..." CFGS="get256 zipf post"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-cfg}
for c in ${CFGS:-get256}; do
for lw in ${LIBS_WAVES}; do
  l=${lw%%:*}; w=${lw##*:}
  RHP_LIB=$PWD/libreactorng_amd/$l.so RHP_WAVES=$w timeout -k 10 180 python bench.py --no-cpu --steps 30 --warmup 5 --config $c > gpurun_out/${TAG}_${l}_w${w}_$c.json 2>gpurun_out/${TAG}_${l}_w${w}_$c.err || exit 1
  echo "$c $l waves=$w $(python -c "import json;d=json.load(open('gpurun_out/${TAG}_${l}_w${w}_$c.json'));print(d['value'],d['roofline']['kernel_ms'],d['config']['ok_fraction'])")"
done; done
