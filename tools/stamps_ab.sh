#!/bin/bash
# stamps (per-section cycle sums) for several RHP_STAMPS builds: "lib:config" pairs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for lc in ${LIBS_CFG}; do
  l=${lc%%:*}; c=${lc##*:}
  RHP_STAMPS_LIB=$PWD/libreactorng_amd/$l.so RHP_WAVES=${STAMP_WAVES:-16} timeout -k 10 200 python tools/stamps.py $c > gpurun_out/stamps_${l}_c$c.txt 2>&1 || exit 1
  echo "== $l config $c"; grep -v amdgpu.ids gpurun_out/stamps_${l}_c$c.txt
done
