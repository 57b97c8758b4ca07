#!/bin/bash
# round 5 session af: state-row strides 276 / 284 (bank offset 5 / 7 per row) against 268
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5ag && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
for r in 1 2; do
  for v in cur s276 s284; do
    for c in get256 zipf post; do
      RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5ag/${c}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r5ag/${c}_$v.json')); print('$v', '$c', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5ag/ab.txt
    done
  done
done
echo SESSION_OK
