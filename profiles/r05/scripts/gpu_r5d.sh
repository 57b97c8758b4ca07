#!/bin/bash
# round 5 session d: the gap between a window's landing and the next window's issue (refill after the
# loads: rl; and that gap at the top issue priority: gp) against pl; stamps of rl; reactor timeline with
# the submit split; parity of the tree
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5d && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
ab() {   # name lib layouts-env
  RHP_LIB=$L/librhp_x_$2.so RHP_BENCH_LAYOUTS=$3 timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --extra-steps 15 \
    > gpurun_out/r5d/ab_$1.json 2>/dev/null || { echo "FAIL $1"; return 1; }
  python3 - gpurun_out/r5d/ab_$1.json $1 >> gpurun_out/r5d/ab.txt <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d.get("extra_configs", {})
k = lambda c: e.get(c, {}).get("roofline", {}).get("kernel_ms", 0) * 1e3
print(f"{sys.argv[2]:8s} c2 {d['roofline']['kernel_ms']*1e3:6.1f} us wall {d['ms_per_step']*1e3:6.1f} us  c3 {k('zipf'):6.1f}  c5 {k('post'):6.1f}  "
      f"chunked {k('chunked'):7.1f}  parity {sorted(set(v if isinstance(v, str) else v.get('result') for v in d.get('parity', {}).values()))}")
PY
}
C="post=compact,chunked=compact"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5d/pytest_parity.log 2>&1 \
 && echo PARITY_OK && tail -1 gpurun_out/r5d/pytest_parity.log \
 && for r in 1 2; do ab pl pl $C && ab rl rl $C && ab gp gp $C || exit 1; done && cat gpurun_out/r5d/ab.txt \
 && RHP_LIB=$L/librhp_x_stampsrl.so STAMPS_CFG=2,3 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5d/stamps_rl.txt 2>&1 && echo STAMPS_OK \
 && RHP_REACTOR_PARSER=gpu RHP_REACTOR_STATS=2 timeout -k 10 120 libreactorng_amd/bin/burst_test 64 64 7 > gpurun_out/r5d/timeline_4k.txt 2>&1 && echo TL_OK && cat gpurun_out/r5d/timeline_4k.txt | grep -v "^load\|^burst"
