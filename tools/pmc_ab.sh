#!/bin/bash
# One PMC pass (instruction mix) per library, config 2: A/B of kernel variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-pmcab}
for l in ${LIBS}; do
  RHP_LIB=$PWD/libreactorng_amd/$l.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
    --output-format csv -d gpurun_out/${TAG}_$l -o p -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-e2e --copies 4 ${BENCH_ARGS} > gpurun_out/${TAG}_$l.log 2>&1 || exit 1
  python3 - "gpurun_out/${TAG}_$l" "$l" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "rhp_dfa" in r.get("Kernel_Name", "")]
acc = collections.defaultdict(float); disp = set()
for r in rows:
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
n = max(len(disp), 1)
print(sys.argv[2], " ".join(f"{k}={v / n / 1e6:.2f}M" for k, v in sorted(acc.items())))
PY
done
