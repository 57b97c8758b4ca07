"""profiles/pmc_traffic.json from a gpu_session.sh PMC step (rocprofv3 --pmc
FETCH_SIZE and WRITE_SIZE, separate passes, per config).

FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md HBM/rocprofv3 section); both counters are per rhp_dfa_kernel
dispatch, averaged over the dispatches of the pass.  They count the L2's
fabric-side requests, Infinity Cache hits included.

usage: python tools/pmc_traffic.py <gpurun_out dir> <TAG> <profiles dir for the copies>
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

def per_dispatch(path):
    acc = defaultdict(float)
    for row in csv.DictReader(open(path)):
        if "rhp_dfa_kernel" in row.get("Kernel_Name", ""):
            acc[row["Dispatch_Id"]] += float(row["Counter_Value"])
    v = list(acc.values())
    return sum(v) / len(v) if v else None


def main():
    out_dir, tag, prof = sys.argv[1], sys.argv[2], sys.argv[3]
    res = {}
    for cfg in ("get256", "zipf", "post", "chunked"):
        f = glob.glob(os.path.join(out_dir, f"pmc_{tag}_{cfg}_FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True)
        w = glob.glob(os.path.join(out_dir, f"pmc_{tag}_{cfg}_WRITE_SIZE", "**", "*counter_collection.csv"), recursive=True)
        if not f or not w:
            continue
        fetch_kb, write_kb = per_dispatch(f[0]), per_dispatch(w[0])
        os.makedirs(prof, exist_ok=True)
        shutil.copy(f[0], os.path.join(prof, f"pmc_{cfg}_FETCH_SIZE.csv"))
        shutil.copy(w[0], os.path.join(prof, f"pmc_{cfg}_WRITE_SIZE.csv"))
        res[cfg] = {
            "hbm_bytes_per_launch": int(fetch_kb * 2048 + write_kb * 1024),
            "fetch_bytes_raw": int(fetch_kb * 1024),
            "fetch_bytes_x2_gfx950": int(fetch_kb * 2048),
            "write_bytes": int(write_kb * 1024),
            "source": f"{prof}/pmc_{cfg}_{{FETCH,WRITE}}_SIZE.csv: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate "
                      f"passes over bench.py --config {cfg} --steps 6; FETCH_SIZE x2 (gfx950), WRITE_SIZE as is; mean per "
                      "rhp_dfa_kernel dispatch; L2 fabric-side requests (Infinity Cache hits included)",
        }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import hashlib
    lib = os.path.join(root, "libreactorng_amd", "librhp.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    for v in res.values():
        v["library_sha256"] = sha   # bench.py flags the numbers stale when the library it runs differs
    json.dump(res, open(os.path.join(root, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
