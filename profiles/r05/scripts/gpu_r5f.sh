#!/bin/bash
# round 5 session f: H2D probe with the reactor's allocation sequence; fair priority rotation A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5f && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
timeout -k 10 120 tools/h2d_probe 2>&1 | head -12 | tee gpurun_out/r5f/h2d_fresh.txt
for v in pl fair pl fair; do
  RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config get256 --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5f/c2_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r5f/c2_$v.json')); print('$v', round(d['roofline']['kernel_ms']*1e3,1), 'us', round(d['ms_per_step']*1e3,1), d['parity'])" | tee -a gpurun_out/r5f/ab.txt
done
