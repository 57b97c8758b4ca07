"""Same-box, same-process A/B of several librhp.so builds on one bench workload.

Every library is loaded side by side (ctypes, RTLD_LOCAL) into one process and
launched on the same rotated device copies of the workload (one set per record
layout: tag=path@layout), round-robin over the libraries R times, K back-to-back
launches per turn timed with HIP events on the launch stream (bench.py's
clock).  Each library's canonical records after its last launch must equal the
first library's (the same digest): an A/B of equal outputs.

  python tools/ab_libs.py --config get256 --rounds 5 --steps 30 \
      cur=libreactorng_amd/librhp.so r4=libreactorng_amd/librhp_x_r4.so
Prints one line per library: median / min / max us per launch over the rounds.
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libreactorng_amd as rhp  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="get256", choices=sorted(bench.CONFIGS))
    ap.add_argument("--layout", default=None, help="request|header|compact (default: the bench's auto layout)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--no-parity", action="store_true", help="diagnostic builds whose records differ")
    ap.add_argument("libs", nargs="+", help="tag=path")
    a = ap.parse_args()
    import torch
    rhp.lib()   # torch's HIP runtime first (one runtime per process)
    cfg = bench.CONFIGS[a.config]
    n = cfg["per_gpu"]
    buf, off = rhp.generate(cfg["gen"], n, cfg["seed"], lo=0)
    sets = {}   # layout -> rotated device copies sharing one set of outputs

    def copies_for(layout):
        if layout not in sets:
            cs = [rhp.DeviceBatch(buf, off, cfg["maxh"], cfg["mode"], layout=layout) for _ in range(a.copies)]
            for c in cs[1:]:
                c.reqs, c.hdrs, c.http = cs[0].reqs, cs[0].hdrs, cs[0].http
            sets[layout] = (cs, [c.desc() for c in cs])
        return sets[layout]
    pristine = None
    libs = []
    for spec in a.libs:   # tag=path[@layout]: a library, and the record layout it is launched with
        tag, path = spec.split("=", 1)
        path, _, lay = path.partition("@")
        layout = bench.LAYOUTS[lay or a.layout or cfg["layout"]]
        L = ctypes.CDLL(os.path.abspath(path))
        L.rhp_parse_batch.argtypes = [ctypes.POINTER(rhp.Batch), ctypes.c_void_p]
        L.rhp_parse_batch.restype = ctypes.c_int
        libs.append((tag, L, layout))
        copies_for(layout)
        if cfg.get("rewrites") and pristine is None:
            pristine = sets[layout][0][0].bytes.clone()
    rhp.check_one_hip_runtime()
    s = torch.cuda.current_stream()

    def launch(L, layout, k):
        copies, descs = sets[layout]
        if pristine is not None:
            copies[k % len(copies)].bytes.copy_(pristine)
        rc = L.rhp_parse_batch(ctypes.byref(descs[k % len(copies)]), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"rhp_parse_batch {rc}")

    ref = None
    for tag, L, layout in libs:   # warm-up and parity (canonical records) against the first library
        c0 = sets[layout][0][0]
        for t in (c0.reqs, c0.hdrs, c0.http):
            t.fill_(0xFF)
        for k in range(4):
            launch(L, layout, k)
        torch.cuda.synchronize()
        res = c0.result()
        out = rhp.record_digest(*rhp.canonical(res, cfg["mode"]))
        if pristine is not None:   # de-framed bytes too: copy 0 restored, launched once more, hashed
            import hashlib
            c0.bytes.copy_(pristine)
            rc = L.rhp_parse_batch(ctypes.byref(sets[layout][1][0]), ctypes.c_void_p(s.cuda_stream))
            torch.cuda.synchronize()
            if rc != 0:
                raise RuntimeError(f"rhp_parse_batch {rc}")
            out = (out, hashlib.sha256(c0.bytes.cpu().numpy().tobytes()).hexdigest())
        if ref is None:
            ref = out
        same = out == ref
        print(f"ab parity {tag}: {'match' if same else 'DIFFERS'}", flush=True)
        if not same and not a.no_parity:
            sys.exit(3)
    times = {tag: [] for tag, _, _ in libs}
    for r in range(a.rounds):
        for tag, L, layout in libs:
            if pristine is not None:
                # a rewriting config restores its bytes before each launch: time each launch
                # alone (events around the kernel only), so the restore copies stay outside
                tot = 0.0
                for k in range(a.steps):
                    copies, descs = sets[layout]
                    copies[(k + 1) % len(copies)].bytes.copy_(pristine)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    rc = L.rhp_parse_batch(ctypes.byref(descs[(k + 1) % len(copies)]), ctypes.c_void_p(s.cuda_stream))
                    e1.record(s)
                    if rc != 0:
                        raise RuntimeError(f"rhp_parse_batch {rc}")
                    torch.cuda.synchronize()
                    tot += e0.elapsed_time(e1)
                times[tag].append(1e3 * tot / a.steps)
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            launch(L, layout, 0)
            e0.record(s)
            for k in range(a.steps):
                launch(L, layout, k + 1)
            e1.record(s)
            torch.cuda.synchronize()
            times[tag].append(1e3 * e0.elapsed_time(e1) / a.steps)
        print(f"ab round {r} " + " ".join(f"{t}={v[-1]:.1f}" for t, v in times.items()), flush=True)
    for tag, v in times.items():
        print(f"ab {a.config} {tag:10s} median {statistics.median(v):7.2f} us  min {min(v):7.2f}  max {max(v):7.2f}"
              f"  ({len(v)} rounds x {a.steps} launches)", flush=True)


if __name__ == "__main__":
    main()
