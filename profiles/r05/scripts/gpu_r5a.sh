#!/bin/bash
# round 5 session a: GPU parity of the tree (new decode, compact http records), A/B of the kernel
# variants (committed base, row stride 260, new decode, new decode + stride, compact http records for
# configs 5 and chunked), stamps of the committed kernel and of the new decode
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5a && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
ab() {   # name lib layouts-env
  RHP_LIB=$L/librhp_x_$2.so RHP_BENCH_LAYOUTS=$3 timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 30 --warmup 5 --extra-steps 15 \
    > gpurun_out/r5a/ab_$1.json 2>/dev/null || { echo "FAIL $1"; return 1; }
  python3 - gpurun_out/r5a/ab_$1.json $1 >> gpurun_out/r5a/ab.txt <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); e = d.get("extra_configs", {})
k = lambda c: e.get(c, {}).get("roofline", {}).get("kernel_ms", 0) * 1e3
print(f"{sys.argv[2]:8s} c2 {d['roofline']['kernel_ms']*1e3:6.1f} us wall {d['ms_per_step']*1e3:6.1f} us  c3 {k('zipf'):6.1f}  c5 {k('post'):6.1f}  "
      f"chunked {k('chunked'):7.1f}  parity {sorted(set(v if isinstance(v, str) else v.get('result') for v in d.get('parity', {}).values()))}")
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest_parity.log 2>&1 \
  && echo PARITY_OK && tail -2 gpurun_out/r5a/pytest_parity.log \
  && ab base base "" && ab s260 s260 "" && ab dx dx "" && ab dxs dxs "" && ab cx cx "post=compact,chunked=compact" \
  && ab pl pl "post=compact,chunked=compact" && ab cf2 cf2 "post=compact,chunked=compact" && ab cf2s cf2s "post=compact,chunked=compact" \
  && ab dx dx "" && ab cf2s cf2s "post=compact,chunked=compact" && ab pl pl "post=compact,chunked=compact" \
  && cat gpurun_out/r5a/ab.txt \
  && RHP_LIB=$L/librhp_x_stamps.so STAMPS_CFG=2,3,5 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5a/stamps_committed.txt 2>&1 \
  && RHP_LIB=$L/librhp_x_stampsdx.so STAMPS_CFG=2,3,5 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5a/stamps_dx.txt 2>&1 \
  && RHP_LIB=$L/librhp_x_stampspl.so STAMPS_CFG=2,5 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5a/stamps_pl.txt 2>&1 && echo STAMPS_OK
