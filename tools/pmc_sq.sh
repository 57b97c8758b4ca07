#!/bin/bash
# Two SQ counter passes (issue/wait split, instruction mix, LDS conflicts) of
# rhp_dfa_kernel on one config, one rocprofv3 run per pass.
# usage: TAG=x CONFIG=get256 [RHP_LIB=...] bash tools/pmc_sq.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-sq}
C=${CONFIG:-get256}
[ -n "$LIST" ] && { timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true; }
run() { # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$name -o p \
    -- python3 bench.py --config $C --extra none --steps 4 --warmup 1 --no-cpu --no-e2e ${BENCH_ARGS} > gpurun_out/${TAG}_$name.log 2>&1
}
run sqa SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
 && run sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES \
 && python3 - gpurun_out/${TAG} <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "_sq*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "rhp_dfa" in r.get("Kernel_Name", ""):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, k), v in per.items():
        acc[k].append(v)
m = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(m):
    print(f"{k:24s} {m[k]:16.0f}")
w = m.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
        print(f"{k:24s} / wave cycles = {m.get(k, 0) / w:.3f}")
if m.get("SQ_LDS_IDX_ACTIVE"):
    print("lds conflict frac", m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"])
PY
