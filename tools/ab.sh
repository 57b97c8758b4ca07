#!/bin/bash
# interleaved A/B: for each config, REPS rounds of (lib1, lib2, ...) -> medians
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-ab}; REPS=${REPS:-3}
for c in ${CFGS:-get256}; do
  for r in $(seq $REPS); do
    for l in ${LIBS}; do
      RHP_LIB=$PWD/libreactorng_amd/$l.so RHP_WAVES=${WAVES:-16} timeout -k 10 120 python bench.py --no-cpu --steps ${STEPS:-30} --warmup 5 --config $c > gpurun_out/${TAG}_${l}_${c}_$r.json 2>/dev/null || exit 1
    done
  done
  for l in ${LIBS}; do
    python - "$TAG" "$l" "$c" "$REPS" <<'PY'
import json, sys, statistics
tag, l, c, reps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
v = [json.load(open(f"gpurun_out/{tag}_{l}_{c}_{r}.json")) for r in range(1, reps + 1)]
g = [d["value"] for d in v]; k = [d["roofline"]["kernel_ms"] for d in v]
print(f"{c:7s} {l:16s} median {statistics.median(g):8.1f} GiB/s  kernel {statistics.median(k)*1000:7.1f} us  all {' '.join('%.0f' % x for x in g)}")
PY
  done
done
