#!/bin/bash
# round 5 session v: the prologue barrier before each wave's first issue (bf) against after it (cur)
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5v && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
for r in 1 2 3; do
  for v in cur bf; do
    for c in get256 post; do
      RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5v/${c}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r5v/${c}_$v.json')); print('$v', '$c', round(d['roofline']['kernel_ms']*1e3,1), 'us', round(d['ms_per_step']*1e3,1), d['parity'])" | tee -a gpurun_out/r5v/ab.txt
    done
  done
done
echo SESSION_OK
