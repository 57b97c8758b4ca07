#!/bin/bash
# round 5 session o: after line windows config 3 is bound by the walk's LDS chain (52 % of LDS cycles are bank
# conflicts): conflict-free code form / row stride, fewer walking waves for uneven ranges
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5o && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
one() {  # lib config
  RHP_LIB=$L/librhp_x_$1.so timeout -k 10 300 python bench.py --config $2 --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5o/$2_$1.json 2>/dev/null || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/r5o/$2_$1.json')); print('$1', '$2', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5o/ab.txt
}
for r in 1 2; do
  for v in cur s260 cf2 cf2s uw11 uw10; do one $v zipf || exit 1; done
  for v in cur s260 cf2s; do one $v get256 && one $v post || exit 1; done
done
echo SESSION_OK
