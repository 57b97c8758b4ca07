#!/bin/bash
# round 5 session ad: issue priority in the loop -- rotation (cur), none (p4), static younger-higher (p1)
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5ad && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
for r in 1 2; do
  for v in cur p4 p1; do
    for c in get256 zipf post; do
      RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5ad/${c}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r5ad/${c}_$v.json')); print('$v', '$c', round(d['roofline']['kernel_ms']*1e3,1), 'us', round(d['ms_per_step']*1e3,1), d['parity'])" | tee -a gpurun_out/r5ad/ab.txt
    done
  done
done
echo SESSION_OK
