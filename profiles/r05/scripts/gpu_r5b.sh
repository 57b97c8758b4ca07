#!/bin/bash
# round 5 session b: stamps (inlined diagnostics) of the phase-locked kernel, config 5 record layouts
# with the lock, line-window diagnostic (time + FETCH of config 3), SQ counters per config, reactor timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5b && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
ab() {   # name lib layouts-env
  RHP_LIB=$L/librhp_x_$2.so RHP_BENCH_LAYOUTS=$3 timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --extra-steps 15 \
    > gpurun_out/r5b/ab_$1.json 2>/dev/null || { echo "FAIL $1"; return 1; }
  python3 - gpurun_out/r5b/ab_$1.json $1 >> gpurun_out/r5b/ab.txt <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d.get("extra_configs", {})
k = lambda c: e.get(c, {}).get("roofline", {}).get("kernel_ms", 0) * 1e3
print(f"{sys.argv[2]:8s} c2 {d['roofline']['kernel_ms']*1e3:6.1f} us wall {d['ms_per_step']*1e3:6.1f} us  c3 {k('zipf'):6.1f}  c5 {k('post'):6.1f}  "
      f"chunked {k('chunked'):7.1f}  parity {sorted(set(v if isinstance(v, str) else v.get('result') for v in d.get('parity', {}).values()))}")
PY
}
RHP_LIB=$L/librhp_x_stampspl.so STAMPS_CFG=2,3,5 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5b/stamps_pl.txt 2>&1 && echo STAMPS_OK && head -14 gpurun_out/r5b/stamps_pl.txt \
 && ab plh pl "" && ab plc pl "post=compact,chunked=compact" && ab plh pl "" && ab plc pl "post=compact,chunked=compact" && cat gpurun_out/r5b/ab.txt || exit 1
for v in pl ladiag; do
  RHP_LIB=$L/librhp_x_$v.so RHP_BENCH_DIAG=1 timeout -k 10 300 python bench.py --config zipf --extra none --no-cpu --no-e2e --steps 30 --warmup 5 \
    > gpurun_out/r5b/zipf_$v.json 2>/dev/null || exit 1
  RHP_LIB=$L/librhp_x_$v.so RHP_BENCH_DIAG=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5b/pmc_${v}_zipf -o p \
    -- python3 bench.py --config zipf --extra none --steps 6 --warmup 2 --no-cpu --no-e2e > gpurun_out/r5b/pmc_${v}_zipf.log 2>&1 || exit 1
done && echo LADIAG_OK \
 && for c in get256 zipf post chunked; do TAG=r5b/sq_$c CONFIG=$c RHP_LIB=$L/librhp_x_pl.so bash tools/pmc_sq.sh > gpurun_out/r5b/sq_$c.txt 2>&1 || exit 1; done && echo SQ_OK \
 && timeout -k 10 600 bash tools/reactor_timeline.sh > gpurun_out/r5b/reactor_timeline.txt 2>&1 && echo TIMELINE_OK
