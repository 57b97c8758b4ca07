"""Summarise rocprofv3 --pmc passes (tools/pmc_probe.sh) for rhp_dfa_kernel.

usage: python tools/pmc_summary.py gpurun_out/<TAG> [out.json] [--steps-per-dispatch BYTES]
Reads <TAG>_{sq1,sq2,sq3,fetch,write}/p_counter_collection.csv, averages each
counter over the kernel's dispatches and derives per-step rates.  FETCH_SIZE is
reported raw and x2 (gfx950 correction, MI355X_MICROARCH.md HBM/rocprofv3
section); WRITE_SIZE raw.  Both are in KiB per the counter definition.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(prefix, kernel="rhp_dfa_kernel"):
    vals = defaultdict(list)
    for path in sorted(glob.glob(prefix + "_*/p_counter_collection.csv")):
        per = defaultdict(float)
        for row in csv.DictReader(open(path)):
            if kernel not in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (_, name), v in per.items():
            vals[name].append(v)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def derive(m, step_bytes):
    d = {}
    g = lambda k: m.get(k, 0.0)
    if g("SQ_WAVE_CYCLES"):
        d["wait_any_frac"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
        d["wait_inst_frac"] = g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")
        d["active_frac"] = g("SQ_ACTIVE_INST_ANY") / g("SQ_WAVE_CYCLES")
    if step_bytes:
        wave_steps = step_bytes / 64.0
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if k in m:
                d[k.lower().replace("sq_insts_", "") + "_per_wave_step"] = m[k] / wave_steps
    if g("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict_frac"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    if "FETCH_SIZE" in m:
        d["fetch_bytes_raw"] = m["FETCH_SIZE"] * 1024
        d["fetch_bytes_x2_gfx950"] = m["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in m:
        d["write_bytes"] = m["WRITE_SIZE"] * 1024
    if "fetch_bytes_x2_gfx950" in d and "write_bytes" in d:
        d["hbm_traffic_bytes"] = d["fetch_bytes_x2_gfx950"] + d["write_bytes"]
    return d


if __name__ == "__main__":
    prefix = sys.argv[1]
    step_bytes = 0.0
    if "--steps-per-dispatch" in sys.argv:
        step_bytes = float(sys.argv[sys.argv.index("--steps-per-dispatch") + 1])
    m = load(prefix)
    out = {"per_dispatch_mean": m, "derived": derive(m, step_bytes)}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 2 and not sys.argv[2].startswith("--"):
        open(sys.argv[2], "w").write(s)
    print(s)
