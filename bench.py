#!/usr/bin/env python3
"""bench.py -- device-resident batched HTTP/1.1 request parse throughput.

Metric (BASELINE.json): "GiB/s device-resident batched HTTP/1.1 request parse,
1/2/4/8 MI355X".  One step = one rhp_parse_batch launch (include/rhp.h) over one
batch of synthetic requests already resident in HBM.

Workloads:
  N=1  config 2: 1M x 256 B GET, 4 headers, max_headers 16 (phr mode) -> `value`;
       configs 3 and 5 and a chunked-body config are
       timed too, in `extra_configs`
  N>1  config 4: config 2's generator sharded evenly, 1M requests per GPU
       (8M at N=8), no collective on the data path -> weak scaling

Launch: `python bench.py --gpus N` starts N rank processes itself (one per GPU,
before any GPU call, device = LOCAL_RANK); under torch.distributed.run the ranks
come from RANK / LOCAL_RANK / WORLD_SIZE, which must equal --gpus.

Inputs rotate over >= 4 resident copies (>= 1 GiB) so every launch reads HBM,
not the 256 MiB Infinity Cache.  value = algorithmic bytes (header-section bytes
the reference reads) of all ranks / max-over-ranks time, GiB/s.

The roofline leg times the kernel with HIP events on the stream it is launched
on (torch's current stream is passed to the C-ABI).  cpu_baseline times the
reference's own parser (oracle/_ref/libref.so: the reference compiled from
/root/reference in the dev container; it travels to the GPU box as a built
library) on rank 0, N=1 only, on a bounded sample of each workload, at 1
thread and at all CPUs this process may use.

--device cpu runs the same harness with the CPU emulation of the kernel
(rhp_emu_parse_batch) instead of the GPU: a test of the launcher, sharding and
reduction on machines without a GPU, never a measurement.
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import libreactorng_amd as rhp  # noqa: E402

LAYOUTS = {"request": rhp.LAYOUT_REQUEST_MAJOR, "header": rhp.LAYOUT_HEADER_MAJOR, "compact": rhp.LAYOUT_COMPACT,
           "dense": rhp.LAYOUT_DENSE, "dense_rm": rhp.LAYOUT_DENSE_RM}
METRIC = "GiB/s device-resident batched HTTP/1.1 request parse, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E, GB/s (MI355X_MICROARCH.md chip table)
CONFIGS = {
    "get256": dict(gen=rhp.GEN_GET256, seed=0x5EED0002, maxh=16, mode=rhp.MODE_PHR, per_gpu=1 << 20,
                   layout="dense",
                   name="config2/4: 1M x 256 B GET, 4 headers per GPU (phr_parse_request, max_headers 16)"),
    "zipf": dict(gen=rhp.GEN_ZIPF, seed=0x5EED0003, maxh=32, mode=rhp.MODE_PHR, per_gpu=1 << 20,
                 layout="dense_rm",
                 name="config3: 1M mixed 64 B-4 KiB Zipf requests, 0-32 headers (max_headers 32)"),
    "post": dict(gen=rhp.GEN_POST1K, seed=0x5EED0005, maxh=16, mode=rhp.MODE_HTTP, per_gpu=1 << 20,
                 layout="dense",
                 name="config5: 1M x 1 KiB POST, Content-Length body skip, 5% malformed (http_read_request)"),
    # not a BASELINE config: the chunked body framing of http_read_request (http.c:73-160, 221-230),
    # SURVEY.md §8f row 3; the bodies are de-framed in place, so every launch starts from restored bytes
    "chunked": dict(gen=rhp.GEN_CHUNKED, seed=0x5EED0006, maxh=16, mode=rhp.MODE_HTTP, per_gpu=1 << 20,
                    layout="header", rewrites=True,
                    name="chunked: 1M x ~1 KiB POST, Transfer-Encoding: chunked (1-8 chunks), de-framed in place, "
                         "5% malformed framing (http_read_request)"),
}


EXTRA_KEYS = ("zipf", "post", "chunked")   # timed beside config 2 at N=1 (extra_configs)


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous request range of one rank."""
    return n_total * rank // world, n_total * (rank + 1) // world


def traffic_from_profile(config_key: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this
    kernel (profiles/pmc_traffic.json: FETCH_SIZE x 2 on gfx950 + WRITE_SIZE),
    the profile it came from, and whether that profile was taken on the library
    this run loads (its sha256); (None, None, False) if absent."""
    import hashlib
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path)).get(config_key, {})
        lib = os.environ.get("RHP_LIB", os.path.join(ROOT, "libreactorng_amd", "librhp.so"))
        match = d.get("library_sha256") == hashlib.sha256(open(lib, "rb").read()).hexdigest()
        if not match:
            print(f"bench.py: profiles/pmc_traffic.json ({config_key}) was not measured on the library this run "
                  f"loads: roofline.traffic is stale", file=sys.stderr)
        return d.get("hbm_bytes_per_launch"), d.get("source"), match
    except Exception:
        return None, None, False


def cpu_info():
    """CPU model and the CPUs this process may use (affinity, cgroup quota)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota)))
    return model, affinity, quota, usable


def cpu_baseline(keys, seconds: float = 5.0, cold_bytes: int = 1 << 30):
    """The reference CPU parser on the host cores, per config, at 1 thread and
    at every usable CPU, over the FULL workload (the config's 1M requests), in
    a memory regime like the GPU's: the batch is replicated until the copies
    hold >= cold_bytes (beyond the host's last-level cache) and the passes
    rotate over the copies, so every pass reads DRAM, as every GPU launch reads
    HBM.  Threads parse contiguous shards of a pass (one pthread per CPU).

    The timed code is the reference's own phr_parse_request (phr configs) or
    http_read_request (config 5), compiled from /root/reference with its -O3
    flags into oracle/_ref/libref.so by oracle/Makefile in the dev container
    (kind "reference").  Without that library the from-scratch restatement
    oracle/liboracle.so is timed instead (kind "port")."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_util import LIBREF, ORC_HDR, ORC_HTTP, ORC_REQ, oracle
    model, affinity, quota, usable = cpu_info()
    have_ref = os.path.exists(LIBREF)
    ref = ctypes.CDLL(LIBREF) if have_ref else None
    vp, u32, c_int = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    out = {}
    kind = "reference" if have_ref else "port"
    for key in keys:
        cfg = CONFIGS[key]
        n = cfg["per_gpu"]
        buf, off = rhp.generate(cfg["gen"], n, cfg["seed"])
        hb = rhp.header_bytes(cfg["gen"], n, cfg["seed"])
        ncopy = max(1, -(-cold_bytes // buf.nbytes))
        rewrites = bool(cfg.get("rewrites"))
        if rewrites:   # http_dechunk rewrites the bytes: a pass parses a copy restored two passes earlier
            ncopy = max(3, ncopy)
        bufs = [buf] + [buf.copy() for _ in range(ncopy - 1)]
        pristine = buf.copy() if rewrites else None
        chk = ctypes.c_long(0)
        if have_ref:
            fn = ref.ref_http_batch_mt if cfg["mode"] == rhp.MODE_HTTP else ref.ref_phr_batch_mt
            fn.restype = ctypes.c_uint64
            fn.argtypes = [vp, vp, u32, u32, c_int, c_int, vp]
            run = lambda b, t, fn=fn, off=off, cfg=cfg, n=n: fn(b.ctypes.data, off.ctypes.data, n, cfg["maxh"], t, 1,
                                                                ctypes.byref(chk))
            what = ("http_read_request" if cfg["mode"] == rhp.MODE_HTTP else "phr_parse_request") + \
                " of the reference (compiled from /root/reference by oracle/Makefile, gcc -O3 -march=x86-64-v3, " \
                "SSE4.2 path)"
        else:
            o = oracle()
            reqs = np.zeros(n, dtype=ORC_REQ)
            hdrs = np.zeros((n, cfg["maxh"]), dtype=ORC_HDR)
            http = np.zeros(n, dtype=ORC_HTTP)

            def run(b, t, off=off, cfg=cfg, n=n):
                if cfg["mode"] == rhp.MODE_HTTP:
                    t0 = time.perf_counter_ns()
                    o.orc_http_batch(b.ctypes.data, off.ctypes.data, n, cfg["maxh"], reqs.ctypes.data,
                                     hdrs.ctypes.data, http.ctypes.data)
                    return time.perf_counter_ns() - t0
                return o.orc_phr_batch_mt(b.ctypes.data, off.ctypes.data, n, cfg["maxh"], reqs.ctypes.data,
                                          hdrs.ctypes.data, t, 1)
            what = "oracle/rhp_oracle.c restatement (gcc -O3 -march=x86-64-v3)"
        res = {}
        for t in sorted({1, usable}):
            if kind == "port" and cfg["mode"] == rhp.MODE_HTTP and t > 1:
                continue
            run(bufs[-1], t)   # warm-up pass (threads, page tables), then rotate from the copy touched longest ago
            if rewrites:
                for b in bufs[:2]:
                    np.copyto(b, pristine)
            ns, passes = 0, 0
            while passes < 2 or ns < seconds / 2 * 1e9:
                if rewrites:   # untimed: the timed span is inside run()
                    np.copyto(bufs[(passes + 2) % ncopy], pristine)
                ns += run(bufs[passes % ncopy], t)
                passes += 1
            res[t] = (hb * passes / (ns / 1e9) / 2 ** 30, passes)
        top = max(res)
        out[key] = {"value": round(res[top][0], 3), "cores": top, "value_1_thread": round(res[1][0], 3),
                    "passes": res[top][1], "copies": ncopy,
                    "sample": f"{what}; the full config, {n} requests of {cfg['name']} "
                              f"({buf.nbytes / 2 ** 20:.0f} MiB), {ncopy} copies rotated "
                              f"({ncopy * buf.nbytes / 2 ** 20:.0f} MiB, beyond the host LLC: each pass reads DRAM), "
                              f"{res[top][1]} passes at {top} threads"}
        del bufs, buf
        gc.collect()
    main_key = keys[0]
    line = {"value": out[main_key]["value"], "unit": "GiB/s", "cores": out[main_key]["cores"], "kind": kind,
            "value_1_thread": out[main_key]["value_1_thread"], "sample": out[main_key]["sample"],
            "memory_regime": "DRAM (full workload, copies rotated beyond the LLC), like the GPU's HBM-resident batches",
            "cpu_model": model, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "per_config": {k: {kk: v for kk, v in d.items() if kk != "sample"} for k, d in out.items()},
            "note": "timed binary: the reference built from its own sources in the dev container "
                    "(oracle/_ref/libref.so), shipped to this box as a library" if kind == "reference" else
                    "timed binary: the from-scratch oracle restatement"}
    return line


# ---------------------------------------------------------------- launcher

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(argv, n: int) -> int:
    """Start n rank processes of this script (before any GPU call here) and
    return the worst exit status.  Rank r drives GPU r (LOCAL_RANK)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


# ---------------------------------------------------------------- timing

class GpuRunner:
    """A config's shard resident in HBM (rotated copies), launched on torch's
    current stream and timed with HIP events on that stream."""

    def __init__(self, cfg, lo, hi, copies, layout, streams=1):
        import hashlib
        import torch
        self.torch = torch
        self.mode = cfg["mode"]
        buf, off = rhp.generate(cfg["gen"], hi - lo, cfg["seed"], lo=lo)
        self.input_sha256 = hashlib.sha256(buf.tobytes()).hexdigest()
        # a config whose launches rewrite the bytes (chunked bodies, http.c:155) restores a copy from
        # this pristine one before it is launched again: >= 3 copies, restored two launches ahead
        self.rewrites = bool(cfg.get("rewrites"))
        if self.rewrites:
            copies = max(3, copies)
        self.copies = [rhp.DeviceBatch(buf, off, cfg["maxh"], cfg["mode"], layout=layout) for _ in range(max(1, copies))]
        self.pristine = self.copies[0].bytes.clone() if self.rewrites else None
        self.nstep = 0
        # one set of output records per stream (batches in flight at once never share outputs)
        self.nstreams = max(1, streams)
        for k, c in enumerate(self.copies):
            o = self.copies[k % self.nstreams]
            c.reqs, c.hdrs, c.http = o.reqs, o.hdrs, o.http
        self.stream = torch.cuda.current_stream()
        self.streams = [self.stream] + [torch.cuda.Stream() for _ in range(self.nstreams - 1)]

    def poison(self):
        """Every output record set filled with 0xFF (outside the timed region): the
        parity check after the timed loop then proves that the timed launches
        wrote the records it hashes."""
        for o in self.copies[:self.nstreams]:
            for t in (o.reqs, o.hdrs, o.http):
                t.fill_(0xFF)
        self.torch.cuda.synchronize()

    def restore_ahead(self):
        """rewriting configs: the copy launched two steps from now gets pristine bytes
        (then >= 2 launches of other bytes lie between its restore and its parse)"""
        if self.rewrites:
            c = self.copies[(self.nstep + 2) % len(self.copies)]
            c.bytes.copy_(self.pristine)

    def step(self, k):
        self.restore_ahead()
        self.copies[self.nstep % len(self.copies)].launch(self.stream)
        self.nstep += 1

    def sync(self):
        self.torch.cuda.synchronize()

    def timed(self, steps):
        """(wall seconds, mean launch ms from HIP events on the launch stream)"""
        torch = self.torch
        if self.rewrites:
            return self.timed_rewriting(steps)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the first record of timing events costs milliseconds on the host: do it outside the timed region
        ev0.record(self.stream)
        ev1.record(self.stream)
        torch.cuda.synchronize()
        gc.collect()
        t0 = time.perf_counter()
        ev0.record(self.stream)
        t1 = time.perf_counter()
        for k in range(steps):
            self.step(k)
        t2 = time.perf_counter()
        ev1.record(self.stream)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if True:   # host-side timing of the timed region, for the record (stderr)
            print(f"bench diag: record {1e3 * (t1 - t0):.3f} ms, {steps} launches {1e3 * (t2 - t1):.3f} ms, "
                  f"record+sync {1e3 * (t3 - t2):.3f} ms", file=sys.stderr)
        return t3 - t0, ev0.elapsed_time(ev1) / steps

    def timed_rewriting(self, steps):
        """A config whose launches rewrite their bytes: each launch is bracketed by
        its own events, the restore of a later copy (a D2D copy of the pristine
        bytes) stays outside them.  (sum of launch seconds, mean launch ms)"""
        torch = self.torch
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        gc.collect()
        for e0, e1 in evs:
            self.restore_ahead()
            e0.record(self.stream)
            self.copies[self.nstep % len(self.copies)].launch(self.stream)
            e1.record(self.stream)
            self.nstep += 1
        torch.cuda.synchronize()
        ms = [e0.elapsed_time(e1) for e0, e1 in evs]
        return sum(ms) * 1e-3, sum(ms) / len(ms)

    def timed_pipelined(self, steps):
        """Wall seconds for `steps` launches, launch k on stream k % S: batch k+1
        starts on the CUs batch k's tail has freed (two batches in flight, as
        the reactor's two batch slots)."""
        torch = self.torch
        start, ends = torch.cuda.Event(), [torch.cuda.Event() for _ in self.streams]
        torch.cuda.synchronize()
        gc.collect()
        t0 = time.perf_counter()
        start.record(self.stream)
        for s in self.streams[1:]:
            s.wait_event(start)
        for k in range(steps):
            self.copies[k % len(self.copies)].launch(self.streams[k % self.nstreams])
        for e, s in zip(ends, self.streams):
            e.record(s)
        for e in ends:
            self.stream.wait_event(e)
        torch.cuda.synchronize()
        self.nstep = steps   # last_result: the outputs of launch steps - 1
        return time.perf_counter() - t0

    def last_result(self):
        """records of the last launch (and, for a rewriting config, its bytes as it left them)"""
        return self.copies[(self.nstep - 1) % len(self.copies)].result()   # its bytes were pristine when launched

    def ok_fraction(self):
        res = self.last_result()
        if res.http is not None:
            return float((res.http["result"] == 1).mean()) if len(res.http) else 1.0
        return float((res.reqs["ret"] > 0).mean()) if len(res.reqs) else 1.0

    def parity(self, spec):
        """The last timed launch's records against the reference's digest of the
        same workload (tests/golden/full_digests.json, made by the compiled
        reference): "match", or a "MISMATCH ..." string."""
        import hashlib
        if spec is None:
            return "unpinned: no reference digest for this shard size"
        if spec["input_sha256"] != self.input_sha256:
            return "MISMATCH: input bytes differ from the ones the reference digest was made on"
        res = self.last_result()
        got = rhp.record_digest(*rhp.canonical(res, self.mode))
        if got != spec["records_sha256"]:
            return f"MISMATCH: records sha256 {got[:16]}... != reference {spec['records_sha256'][:16]}..."
        if "bytes_out_sha256" in spec:   # chunked bodies de-framed in place (http.c:134-160)
            if hashlib.sha256(res.bytes_out.tobytes()).hexdigest() != spec["bytes_out_sha256"]:
                return "MISMATCH: de-framed bytes differ from the reference's"
        return "match"


class EmuRunner:
    """--device cpu: the kernel's CPU emulation (harness tests only)."""

    def __init__(self, cfg, lo, hi, copies, layout):
        self.buf, self.off = rhp.generate(cfg["gen"], hi - lo, cfg["seed"], lo=lo)
        self.cfg = cfg
        self.layout = layout
        self.res = None

    def poison(self):
        self.res = None

    def step(self, k):
        self.res, _ = rhp.emulate(self.buf, self.off, self.cfg["maxh"], self.cfg["mode"], self.layout)

    def sync(self):
        pass

    def timed(self, steps):
        t0 = time.perf_counter()
        for k in range(steps):
            self.step(k)
        wall = time.perf_counter() - t0
        return wall, wall * 1e3 / max(steps, 1)

    def ok_fraction(self):
        return float((self.res.reqs["ret"] > 0).mean()) if self.res is not None and len(self.res.reqs) else 1.0

    def parity(self, spec):
        if spec is None:
            return "unpinned: no reference digest for this shard size"
        got = rhp.record_digest(*rhp.canonical(self.res, self.cfg["mode"]))
        return "match" if got == spec["records_sha256"] else "MISMATCH: records differ from the reference digest"


# reference digests of the timed workloads (tests/golden/full_digests.json, made
# by the reference compiled from /root/reference: tests/golden/make_golden.py)
GOLDEN_DIGESTS = os.path.join(ROOT, "tests", "golden", "full_digests.json")
GOLDEN_NAMES = {"zipf": "config3_zipf_h32", "post": "config5_post1k_http_h16", "chunked": "chunked_post_http_h16"}


def golden_spec(key, lo, n):
    """The reference digest of requests [lo, lo + n) of a config, or None.  Config
    2/4's shards are keyed by their first request (rank r of any N <= 8 parses
    requests [r * 2^20, (r + 1) * 2^20), config 4's shard r)."""
    sets = json.load(open(GOLDEN_DIGESTS))["sets"]
    cfg = CONFIGS[key]
    names = [GOLDEN_NAMES[key]] if key in GOLDEN_NAMES else [f"config4_get256_shard{k}of8" for k in range(8)]
    for name in names:
        s = sets.get(name)
        if s and s["lo"] == lo and s["n"] == n and s["seed"] == cfg["seed"] and s["max_headers"] == cfg["maxh"] \
                and s["mode"] == cfg["mode"] and s["config"] == cfg["gen"]:
            return dict(s, name=name)
    return None


def run_config(key, args, rank, world, per_gpu, steps, warmup, dist, streams=1):
    cfg = CONFIGS[key]
    n_total = per_gpu * world
    lo, hi = shard_range(n_total, rank, world)
    alg_bytes = rhp.header_bytes(cfg["gen"], hi - lo, cfg["seed"], lo=lo)
    # RHP_BENCH_LAYOUTS="post=compact,zipf=request" (A/B runs) overrides a config's layout under --layout auto
    over = dict(kv.split("=") for kv in os.environ.get("RHP_BENCH_LAYOUTS", "").split(",") if "=" in kv)
    lay_name = over.get(key, cfg["layout"]) if args.layout == "auto" else args.layout
    layout = LAYOUTS[lay_name]
    streams = streams if args.device == "gpu" and not cfg.get("rewrites") else 1
    runner = (GpuRunner(cfg, lo, hi, max(args.copies, streams), layout, streams=streams) if args.device == "gpu"
              else EmuRunner(cfg, lo, hi, args.copies, layout))
    for k in range(warmup):
        runner.step(k)
    runner.sync()
    ok_frac = runner.ok_fraction()
    runner.poison()   # the records the parity check hashes are the timed launches' own
    if dist is not None:
        dist.barrier()
    runner.sync()
    wall, kern_ms = runner.timed(steps)
    if dist is not None:
        dist.barrier()
    single = None
    if streams > 1:
        # the same K steps with the batches alternating over `streams` HIP streams: the
        # value's timed region (the single-stream one above gives the kernel time)
        single = wall
        runner.timed_pipelined(warmup)
        runner.poison()
        if dist is not None:
            dist.barrier()
        runner.sync()
        wall = runner.timed_pipelined(steps)
        if dist is not None:
            dist.barrier()
    # outside the timed region: the last timed launch's records against the reference's digest
    spec = golden_spec(key, lo, hi - lo)
    parity = runner.parity(spec)
    parity_entry = {"result": parity, "digest": spec["name"] if spec else None}
    if parity.startswith("MISMATCH"):
        print(f"bench.py: PARITY {key} rank {rank}: {parity}", file=sys.stderr)
    total_alg = float(alg_bytes)
    if dist is not None:
        import torch
        t = torch.tensor([wall, kern_ms, single or 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, kern_ms = float(t[0]), float(t[1])
        single = float(t[2]) if single is not None else None
        tb = torch.tensor([float(alg_bytes)], dtype=torch.float64)
        dist.all_reduce(tb)
        total_alg = float(tb[0])
        # every rank's verdict reaches rank 0's line (0 match, 1 unpinned, 2 mismatch)
        code = 2 if parity.startswith("MISMATCH") else 0 if parity == "match" else 1
        codes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(codes, torch.tensor([code], dtype=torch.int64))
        parity_entry["ranks"] = ["match" if int(c) == 0 else "unpinned" if int(c) == 1 else "MISMATCH" for c in codes]
        if any(int(c) == 2 for c in codes):
            parity_entry["result"] = "MISMATCH on some rank"
        elif any(int(c) == 1 for c in codes):
            parity_entry["result"] = "match on the ranks with a reference digest" if any(int(c) == 0 for c in codes) \
                else parity_entry["result"]
    return dict(cfg=cfg, lo=lo, hi=hi, n_total=n_total, alg_bytes=alg_bytes, total_alg=total_alg, wall=wall,
                kern_ms=kern_ms, ok_frac=ok_frac, steps=steps, warmup=warmup, parity=parity_entry, layout=lay_name,
                streams=streams, single_wall=single)


def roofline(r, key):
    achieved = r["alg_bytes"] / (r["kern_ms"] * 1e-3) / 1e9
    traffic, source, match = traffic_from_profile(key)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": source,
            "traffic_library_match": match,
            "kernel_ms": round(r["kern_ms"], 4), "algorithmic_bytes_per_launch": int(r["alg_bytes"])}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="get256", choices=sorted(CONFIGS))
    ap.add_argument("--extra", default="auto", choices=["auto", "none"],
                    help="auto: at N=1 also time configs 3 and 5 and the chunked config (extra_configs)")
    ap.add_argument("--extra-steps", type=int, default=20)
    ap.add_argument("--extras", default=",".join(EXTRA_KEYS), help="comma list of the extra configs to time")
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--per-gpu", type=int, default=0, help="requests per GPU (default: the config's 1M)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end leg")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams the timed batches of the main config alternate over (`value`): two batches "
                         "in flight, as the reactor's two slots, so one batch's tail overlaps the next one's start; "
                         "1 = one stream.  The single-stream rate and the per-launch kernel time (roofline) are "
                         "measured too, on one stream")
    ap.add_argument("--impl", type=int, default=rhp.IMPL_DFA)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--layout", default="auto", choices=["auto"] + sorted(LAYOUTS),
                    help="header record layout of the batch ABI (include/rhp.h rhp_layout); auto: the "
                         "config's (dense 8-byte request / 2-byte header records for the uniform phr batches of "
                         "configs 2/4 (header-major) and config 3 (request-major: its header counts vary), compact "
                         "records for config 5 (http mode), header-major for the chunked config)")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(argv, args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only: no data-path collective
    if args.device == "gpu":
        import torch
        torch.cuda.set_device(local)
        rhp.lib().rhp_set_impl(args.impl)
    per_gpu = args.per_gpu or CONFIGS[args.config]["per_gpu"]

    r = run_config(args.config, args, rank, world, per_gpu, args.steps, args.warmup, dist, streams=max(1, args.streams))
    extra = {}
    if world == 1 and args.extra == "auto" and args.config == "get256":
        for key in [k for k in args.extras.split(",") if k in EXTRA_KEYS]:
            e = run_config(key, args, rank, world, args.per_gpu or CONFIGS[key]["per_gpu"], args.extra_steps,
                           3, None)
            extra[key] = {"workload": CONFIGS[key]["name"], "value": round(e["total_alg"] / (e["kern_ms"] * 1e-3)
                                                                           / 2 ** 30, 2),
                          "unit": "GiB/s", "steps": e["steps"],
                          # a rewriting config's launches are timed one by one with HIP events (the D2D
                          # restore of its bytes between launches stays outside): no wall time per step
                          ("ms_per_launch_hip_events" if CONFIGS[key].get("rewrites") else "ms_per_step"):
                              round(e["wall"] * 1e3 / e["steps"], 4),
                          "ok_fraction": e["ok_frac"], "record_layout": f"{e['layout']}-major",
                          "parity": e["parity"], "roofline": roofline(e, key)}

    if rank == 0:
        cfg = r["cfg"]
        kernel = (rhp.lib().rhp_kernel_name().decode() if args.device == "gpu"
                  else "rhp_emu_parse_batch (CPU emulation: harness test, not a measurement)")
        line = {
            "metric": METRIC,
            "value": round(r["total_alg"] * r["steps"] / r["wall"] / 2 ** 30, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": r["steps"], "warmup": r["warmup"],
            "ms_per_step": round(r["wall"] * 1e3 / r["steps"], 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": cfg["name"], "requests_per_gpu": r["hi"] - r["lo"], "global_requests": r["n_total"],
                       "algorithmic_bytes_per_gpu": int(r["alg_bytes"]), "resident_copies": args.copies,
                       "max_headers": cfg["maxh"], "parallelism": f"shard{world}", "ok_fraction": r["ok_frac"],
                       "kernel": kernel, "device": args.device, "record_layout": f"{r['layout']}-major"},
            "roofline": roofline(r, args.config),
        }
        # parity of every timed workload: the records of its last timed launch
        # hashed against the reference's digest (GOLDEN_DIGESTS)
        line["parity"] = {("config4" if world > 1 else "config2") if args.config == "get256" else args.config:
                          r["parity"]["result"]}
        line["parity"].update({k: v["parity"]["result"] for k, v in extra.items()})
        line["parity_detail"] = {args.config: r["parity"], **{k: v["parity"] for k, v in extra.items()}}
        line["library_sha256"] = rhp.library_sha256() if args.device == "gpu" else None
        line["batches_in_flight"] = r["streams"]
        if r.get("single_wall") is not None:
            line["single_stream"] = {"value": round(r["total_alg"] * r["steps"] / r["single_wall"] / 2 ** 30, 2),
                                     "ms_per_step": round(r["single_wall"] * 1e3 / r["steps"], 4),
                                     "note": "the same K steps on one HIP stream (one batch at a time)"}
        if extra:
            line["extra_configs"] = extra
        if world == 1 and args.device == "gpu" and not args.no_e2e:
            # north_star: the path starts and ends in host memory; the rate with
            # pinned H2D -> kernel -> records written into mapped host memory,
            # chunked over 3 streams (never `value`, which is device-resident).
            # It runs in a child process of its own, as a receiver would: inside
            # this process (its device copies, streams and allocations) the same
            # pipeline measured 43 GiB/s with H2D alone 5.3 ms, in its own 47.6-48.5
            # with H2D alone 5.08 ms (profiles/r04/final/e2e_in_process_vs_child.txt)
            e2e_cmd = [sys.executable, os.path.join(ROOT, "tools", "e2e_pcie.py"), "--config", args.config,
                       "--n", str(per_gpu), "--reps", "7"]
            try:   # the headline line does not depend on this leg: a failure is recorded, not raised
                p = subprocess.run(e2e_cmd, capture_output=True, text=True, timeout=600)
                if p.returncode != 0:
                    raise RuntimeError(f"exit {p.returncode}: " + p.stderr[-1500:])
                line["e2e"] = json.loads(p.stdout.strip().splitlines()[-1])
                line["e2e"]["process"] = "a child process of bench.py (tools/e2e_pcie.py)"
            except Exception as exc:
                line["e2e"] = {"error": repr(exc)[-2000:]}
                print(f"bench.py: e2e leg failed: {exc!r}", file=sys.stderr)
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline([args.config] + [k for k in EXTRA_KEYS if k in extra])
        print(json.dumps(line), flush=True)
    bad = "MISMATCH" in r["parity"]["result"] or any("MISMATCH" in v["parity"]["result"] for v in extra.values())
    if dist is not None:
        dist.destroy_process_group()
    if bad and not os.environ.get("RHP_BENCH_DIAG"):   # RHP_BENCH_DIAG: diagnostic builds that write wrong records on purpose
        print("bench.py: parity MISMATCH against the reference digest (see the line's parity)", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
