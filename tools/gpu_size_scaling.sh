#!/bin/bash
# Config 2's kernel time and HBM traffic against batch size (VERDICT r3 item 2c:
# the slope from 2M to 4M requests).  Copies are rotated so every launch reads
# past the Infinity Cache (1, 2, 4 GiB of batches).  One stream: the kernel time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
out=gpurun_out/size_scaling_${TAG:-x}.txt; : > $out
for nc in 524288:8 1048576:4 2097152:2 4194304:1 4194304:2; do
  n=${nc%%:*}; c=${nc##*:}
  timeout -k 10 300 python bench.py --per-gpu $n --copies $c --extra none --no-cpu --no-e2e --streams 1 --steps 20 --warmup 5 \
    > gpurun_out/ss_${n}_${c}.json 2>/dev/null || { echo "FAIL $n"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ss_${n}_${c}.json')); print('config2', $n, 'copies', $c, 'kernel_us', round(d['roofline']['kernel_ms']*1e3,1), 'frac', d['roofline']['frac'])" >> $out
done
for n in 1048576 2097152 4194304; do
  for k in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d gpurun_out/ss_pmc_${n}_$k -o p \
      -- python3 bench.py --per-gpu $n --copies $((4194304 / n)) --extra none --steps 6 --warmup 2 --streams 1 --no-cpu --no-e2e \
      > gpurun_out/ss_pmc_${n}_$k.log 2>&1 || { echo "PMC FAIL $n $k"; exit 1; }
  done
  python3 - $n >> $out << 'PY'
import csv, sys
from collections import defaultdict
n = int(sys.argv[1])
def mean(k):
    acc = defaultdict(float)
    for r in csv.DictReader(open(f"gpurun_out/ss_pmc_{n}_{k}/p_counter_collection.csv")):
        if "rhp_dfa_kernel" in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = list(acc.values())
    return sum(v) / len(v)
f, w = mean("FETCH_SIZE") * 2048, mean("WRITE_SIZE") * 1024
print(f"config2 {n} fetch_x2 {f / 1e6:.1f} MB ({f / n:.1f} B/request) write {w / 1e6:.1f} MB ({w / n:.1f} B/request)")
PY
done
cat $out
