#!/usr/bin/env python3
"""bench.py -- device-resident batched HTTP/1.1 request parse throughput.

Metric (BASELINE.json): "GiB/s device-resident batched HTTP/1.1 request parse,
1/2/4/8 MI355X".  One step = one rhp_parse_batch launch (include/rhp.h) over one
batch of synthetic requests already resident in HBM.

Workloads:
  N=1  config 2: 1M x 256 B GET, 4 headers, max_headers 16 (phr mode)
  N>1  config 4: config 2's generator sharded evenly, 1M requests per GPU
       (8M at N=8), no collective on the data path -> weak scaling
  --config zipf|post are the other BASELINE configs (parity-tested; optional lines)

Inputs rotate over >= 4 resident copies (>= 1 GiB) so every launch reads HBM,
not the 256 MiB Infinity Cache.  value = algorithmic bytes (header-section bytes
the reference reads) of all ranks / max-over-ranks time, in GiB/s.

The roofline leg times the kernel with HIP events on the stream it is launched
on (torch's current stream is passed to the C-ABI).  cpu_baseline times the
oracle restatement (oracle/liboracle.so, "port") on rank 0, N=1 only, on a
bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import libreactorng_amd as rhp  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E, GB/s (MI355X_MICROARCH.md chip table)
CONFIGS = {
    "get256": dict(gen=rhp.GEN_GET256, seed=0x5EED0002, maxh=16, mode=rhp.MODE_PHR, per_gpu=1 << 20,
                   name="config2/4: 1M x 256 B GET, 4 headers per GPU (phr_parse_request, max_headers 16)"),
    "zipf": dict(gen=rhp.GEN_ZIPF, seed=0x5EED0003, maxh=32, mode=rhp.MODE_PHR, per_gpu=1 << 20,
                 name="config3: 1M mixed 64 B-4 KiB Zipf requests, 0-32 headers (max_headers 32)"),
    "post": dict(gen=rhp.GEN_POST1K, seed=0x5EED0005, maxh=16, mode=rhp.MODE_HTTP, per_gpu=1 << 20,
                 name="config5: 1M x 1 KiB POST, Content-Length body skip, 5% malformed (http_read_request)"),
}


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous request range of one rank."""
    return n_total * rank // world, n_total * (rank + 1) // world


def traffic_from_profile(config_key: str):
    """HBM bytes per launch from a committed rocprofv3 PMC summary, if any
    (tools/pmc_traffic.py writes it; FETCH_SIZE doubled on gfx950)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        return d.get(config_key, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(cfg, seconds: float = 12.0):
    """The reference CPU parser on the host cores, on a bounded sample of the workload.

    Prefers the real reference (phr_parse_request compiled from the reference's
    sources with its own -O3 flags into oracle/_ref/libref.so by oracle/Makefile,
    kind "reference"); falls back to the from-scratch restatement (kind "port")
    when that library is absent (it is built only where /root/reference exists)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_util import LIBREF, ORC_HDR, ORC_REQ, oracle
    n = 1 << 18
    buf, off = rhp.generate(cfg["gen"], n, cfg["seed"])
    hb = rhp.header_bytes(cfg["gen"], n, cfg["seed"])
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    if os.path.exists(LIBREF):
        ref = ctypes.CDLL(LIBREF)
        ref.ref_phr_batch_mt.restype = ctypes.c_uint64
        ref.ref_phr_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        chk = ctypes.c_long(0)
        run = lambda t, reps: ref.ref_phr_batch_mt(buf.ctypes.data, off.ctypes.data, n, cfg["maxh"], t, reps,
                                                   ctypes.byref(chk))
        kind, what = "reference", ("phr_parse_request of the reference (src/picohttpparser/picohttpparser.c, "
                                   "gcc -O3 -march=x86-64-v3 as its Makefile.am:61 builds it, SSE4.2 path)")
    else:
        o = oracle()
        reqs = np.zeros(n, dtype=ORC_REQ)
        hdrs = np.zeros((n, cfg["maxh"]), dtype=ORC_HDR)
        run = lambda t, reps: o.orc_phr_batch_mt(buf.ctypes.data, off.ctypes.data, n, cfg["maxh"],
                                                 reqs.ctypes.data, hdrs.ctypes.data, t, reps)
        kind, what = "port", "oracle/rhp_oracle.c phr_parse_request restatement (gcc -O3 -march=x86-64-v3)"
    out = {}
    for t in sorted({1, threads}):
        run(t, 1)
        one = run(t, 1) / 1e9
        reps = max(1, int(seconds / 2 / max(one, 1e-6)))
        ns = run(t, reps)
        out[t] = (hb * reps / (ns / 1e9) / 2 ** 30, reps)
    v, reps = out[threads]
    return {"value": round(v, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1_thread": round(out[1][0], 3),
            "sample": f"{what}; {n} requests of the same workload x {reps} passes, {threads} pthreads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="get256", choices=sorted(CONFIGS))
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--impl", type=int, default=rhp.IMPL_DFA)
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = max(world, 1)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only: no data-path collective
    torch.cuda.set_device(local)
    cfg = CONFIGS[args.config]
    lib = rhp.lib()
    lib.rhp_set_impl(args.impl)

    n_total = cfg["per_gpu"] * world
    lo, hi = shard_range(n_total, rank, world)
    buf, off = rhp.generate(cfg["gen"], hi - lo, cfg["seed"], lo=lo)
    alg_bytes = rhp.header_bytes(cfg["gen"], hi - lo, cfg["seed"], lo=lo)
    copies = [rhp.DeviceBatch(buf, off, cfg["maxh"], cfg["mode"]) for _ in range(max(1, args.copies))]
    # the output buffers of copy 0 are shared so records stay in one place
    for c in copies[1:]:
        c.reqs, c.hdrs, c.http = copies[0].reqs, copies[0].hdrs, copies[0].http
    stream = torch.cuda.current_stream()

    def step(k):
        copies[k % len(copies)].launch(stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()

    # sanity: records of this shard are what the template says (cheap, host side)
    res = copies[0].result()
    ok_frac = float((res.reqs["ret"] > 0).mean()) if len(res.reqs) else 1.0

    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        step(k)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    kern_ms = ev0.elapsed_time(ev1) / args.steps   # avg launch duration on the launch stream

    elapsed = wall
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        tb = torch.tensor([float(alg_bytes)], dtype=torch.float64)
        torch.distributed.all_reduce(tb)
        total_alg = float(tb[0])
    else:
        total_alg = float(alg_bytes)

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        value = total_alg * args.steps / elapsed / 2 ** 30
        per_launch = float(alg_bytes)
        achieved = per_launch / (kern_ms * 1e-3) / 1e9
        line = {
            "metric": "GiB/s device-resident batched HTTP/1.1 request parse, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": cfg["name"], "requests_per_gpu": hi - lo, "global_requests": n_total,
                       "algorithmic_bytes_per_gpu": int(alg_bytes), "resident_copies": len(copies),
                       "max_headers": cfg["maxh"], "parallelism": f"shard{world}", "ok_fraction": ok_frac,
                       "kernel": lib.rhp_kernel_name().decode()},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic_from_profile(args.config),
                         "kernel_ms": round(kern_ms, 4)},
        }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
