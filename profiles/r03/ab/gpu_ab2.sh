#!/bin/bash
# A/B of kernel builds (libreactorng_amd/librhp_x_<name>.so): bench.py kernel times of
# configs 2, 3, 5 per build, interleaved over ROUNDS rounds.  usage: LIBS="a b c" ROUNDS=2
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
out=gpurun_out/ab_${TAG:-x}.txt; : > $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for l in $LIBS; do
    RHP_LIB=$PWD/libreactorng_amd/librhp_x_${l%%@*}.so timeout -k 10 300 python bench.py ${BENCH_ARGS} $( [[ $l == *@* ]] && echo --layout ${l##*@} ) --no-cpu --no-e2e --steps 30 --warmup 5 --extra-steps 15 \
      > gpurun_out/ab_$l.json 2>/dev/null || { echo "FAIL $l" >> $out; exit 1; }
    python - "$l" >> $out << 'PY'
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json"))
e = d.get("extra_configs", {})
ss = d.get("single_stream", {}).get("ms_per_step")
print(f"{sys.argv[1]:10s} c2 {d['roofline']['kernel_ms']*1e3:7.1f} us (frac {d['roofline']['frac']:.3f}, wall {d['ms_per_step']*1e3:6.1f} us"
      + f" x{d.get('batches_in_flight', 1)}" + (f", one stream {ss*1e3:6.1f} us" if ss else "") + ")  "
      f"c3 {e.get('zipf', {}).get('roofline', {}).get('kernel_ms', 0)*1e3:7.1f} us  c5 {e.get('post', {}).get('roofline', {}).get('kernel_ms', 0)*1e3:7.1f} us  "
      f"chunked {e.get('chunked', {}).get('roofline', {}).get('kernel_ms', 0)*1e3:7.1f} us  "
      f"ok {d['config']['ok_fraction']:.3f}  parity {sorted(set(d.get('parity', {}).values()))}")
PY
  done
done
cat $out
