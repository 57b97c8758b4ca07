#!/bin/bash
# round 5 session x: config 3 with 13 walking waves (the order keeps the last three waves' staging)
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5x && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
for r in 1 2 3; do
  for v in cur uw13; do
    RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config zipf --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5x/zipf_$v.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r5x/zipf_$v.json')); print('$v', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5x/ab.txt
  done
done
echo SESSION_OK
