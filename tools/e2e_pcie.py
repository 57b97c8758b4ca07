"""End-to-end rate from host memory to host memory (north_star: "this path starts and
ends in host memory -- the io_uring recv buffer").

The batch (config 2 by default: 1M x 256 B) sits in pinned host memory; it is cut
into chunks that stream through S HIP streams (chunk k on stream k mod S; one
stream per engine -- H2D, kernels, D2H -- measured slower: 34-38 GiB/s, the copies
back trailing the last H2D by 0.8-1.8 ms): pinned hipMemcpyAsync H2D of the
chunk's bytes and offsets -> rhp_parse_batch on that chunk (header records
header-major within the chunk: compact 4-byte records in phr mode, rhp.h) -> D2H
of the chunk's request records.  The host reads each chunk's request records as
they land (a consumer needs them first anyway), takes the largest num_headers of
the chunk, and copies back only header rows 0 .. that - 1 on a copy stream of
their own -- the records the requests use, not every one of the max_headers
slots (config 2: 16 + 4 x 4 = 32 B per request, not 16 + 16 x 8), plus the
chunk's wide records when one of its requests took the exact path.  Copies of
one chunk overlap the kernel of another and the two copy directions overlap
each other.

Reports GiB/s of algorithmic bytes over the wall time of the whole batch, next to
the device-resident kernel rate of the same chunks and the copy-only rates, and
the timeline of the fastest end-to-end repetition from HIP events: per copy
direction and for the kernels, the union of their busy intervals, so a slow run
says which engine was busy (or idle) for how long.

usage: python tools/e2e_pcie.py [--config get256] [--chunks 16] [--streams 3] [--reps 5]
"""
import argparse
import gc
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libreactorng_amd as rhp  # noqa: E402
from bench import CONFIGS  # noqa: E402


def _union_ms(spans):
    """total length of the union of [a, b) intervals (ms)"""
    tot, end = 0.0, -1e30
    for a, b in sorted(spans):
        if b <= end:
            continue
        tot += b - max(a, end)
        end = b
    return tot


def chunk_bounds(n, chunks, taper):
    """request bounds of the chunks: equal ones, then `taper` chunks of halving size
    (the last two equal), so the work left after the last H2D -- that chunk's kernel
    and copies back -- is small"""
    taper = min(taper, chunks - 1)
    w = [1.0] * (chunks - taper) + [0.5 ** min(j + 1, taper - 1 if taper > 1 else 1) for j in range(taper)]
    acc, tot, out = 0.0, sum(w), [0]
    for x in w[:-1]:
        acc += x
        out.append(int(n * acc / tot))
    return out + [n]


def numa_diag():
    """Where the host side runs relative to the GPU: the CPU and NUMA node of the
    calling thread, and the GPU's NUMA node (sysfs, by its PCI bus id)."""
    try:
        libc = ctypes.CDLL("libc.so.6")
        cpu = libc.sched_getcpu()
        node = next((int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node")
                     and os.path.exists(f"/sys/devices/system/node/{d}/cpu{cpu}")), None)
        hip = ctypes.CDLL("libamdhip64.so")
        dev = ctypes.c_int()
        hip.hipGetDevice(ctypes.byref(dev))
        bus = ctypes.create_string_buffer(64)
        hip.hipDeviceGetPCIBusId(bus, 64, dev)
        bid = bus.value.decode().lower()
        gpu_node = int(open(f"/sys/bus/pci/devices/{bid}/numa_node").read())
        return {"cpu": cpu, "cpu_node": node, "gpu_pci": bid, "gpu_node": gpu_node,
                "affinity_cpus": len(os.sched_getaffinity(0))}
    except Exception as exc:   # diagnostics only
        return {"error": repr(exc)}


class MappedHost:
    """Pinned host memory the kernel writes directly (hipHostMalloc, mapped): the
    records cross PCIe as the kernel stores them, no D2H copy, no copy engine."""

    def __init__(self, nbytes):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.h, self.d = ctypes.c_void_p(), ctypes.c_void_p()
        assert self.hip.hipHostMalloc(ctypes.byref(self.h), ctypes.c_size_t(max(nbytes, 1)), ctypes.c_uint(0x2)) == 0
        assert self.hip.hipHostGetDevicePointer(ctypes.byref(self.d), self.h, ctypes.c_uint(0)) == 0
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(self.h.value))

    def free(self):
        self.hip.hipHostFree(self.h)


def e2e(config="get256", n=1 << 20, chunks=16, streams=3, reps=5, taper=0, records="host"):
    """The end-to-end measurement as a dict (bench.py's `e2e` object)."""
    args = argparse.Namespace(config=config, n=n, chunks=chunks, streams=streams, reps=reps, taper=taper,
                              records=records)
    cfg = CONFIGS[args.config]
    n, maxh, mode = args.n, cfg["maxh"], cfg["mode"]
    buf, off = rhp.generate(cfg["gen"], n, cfg["seed"])
    alg = rhp.header_bytes(cfg["gen"], n, cfg["seed"])
    dev = torch.device("cuda")
    RS = rhp.REQ_DTYPE.itemsize
    bounds = chunk_bounds(n, args.chunks, args.taper)
    # phr mode: compact records (rhp.h RHP_LAYOUT_COMPACT: a 4-byte record per header, header-major in
    # the chunk, the exact path's requests in the chunk's wide area); http mode: header-major rhp_hdr_t
    layout = rhp.LAYOUT_COMPACT if mode == rhp.MODE_PHR else rhp.LAYOUT_HEADER_MAJOR
    HB = 4 if layout == rhp.LAYOUT_COMPACT else rhp.HDR_DTYPE.itemsize   # bytes per record of a row
    hbase = [0]
    for k in range(args.chunks):
        hbase.append(hbase[-1] + ((rhp.hdrs_bytes(bounds[k + 1] - bounds[k], maxh, layout) + 255) & ~255))

    # pinned host buffers (the recv side) and full-size device mirrors; chunk k's
    # header records are header-major within the chunk: row r of it is one
    # contiguous run of (hi - lo) records at hdr_base(k) + r * (hi - lo) * 8
    # the receive side: pinned host memory from hipHostMalloc (torch's pin_memory
    # blocks, taken inside bench.py's long-running process, copied 5 % slower
    # with idle gaps: H2D alone 5.34 vs 5.09 ms); the copies by hipMemcpyAsync
    numa = numa_diag()
    m_bytes, m_off = MappedHost(buf.nbytes), MappedHost(off.nbytes)
    m_bytes.array[:] = buf
    m_off.array[:] = off.view(np.uint8)
    h_bytes = torch.from_numpy(m_bytes.array)
    h_off = torch.from_numpy(m_off.array.view(np.int64))
    hip = m_bytes.hip
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    zero_copy = args.records == "host"   # the kernel writes the records into mapped host memory
    if zero_copy:
        m_reqs, m_hdrs = MappedHost(n * RS), MappedHost(hbase[-1])
        h_reqs, h_hdrs = torch.from_numpy(m_reqs.array), torch.from_numpy(m_hdrs.array)
    else:
        h_reqs = torch.empty(n * RS, dtype=torch.uint8).pin_memory()
        h_hdrs = torch.zeros(hbase[-1], dtype=torch.uint8).pin_memory()
    d_bytes = torch.empty_like(h_bytes, device=dev)
    d_off = torch.empty_like(h_off, device=dev)
    d_reqs = torch.empty_like(h_reqs, device=dev)
    d_hdrs = torch.empty_like(h_hdrs, device=dev)
    d_http = torch.zeros(max(1, n if mode == rhp.MODE_HTTP else 1) * rhp.HTTP_DTYPE.itemsize,
                         dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream() for _ in range(args.streams)]
    rows_stream = torch.cuda.Stream()   # D2H of header rows, issued as each chunk's request records land
    works = [torch.zeros(rhp.RHP_WORK_WORDS, dtype=torch.int32, device=dev) for _ in streams]
    lib = rhp.lib()
    reqs_view = h_reqs.numpy().view(rhp.REQ_DTYPE)
    EV = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731

    def run(do_h2d=True, do_kernel=True, do_d2h=True, timeline=None):
        t0 = EV()
        t0.record(streams[0])
        for s in streams[1:] + [rows_stream]:
            s.wait_event(t0)
        marks = []   # per chunk: (h2d start, h2d end, kernel end, reqs end) events
        for k in range(args.chunks):
            lo, hi = bounds[k], bounds[k + 1]
            s = streams[k % len(streams)]
            b0, b1 = int(off[lo]), min(int(off[hi]) + rhp.RHP_PAD, buf.size)   # + the pad the ABI reads
            e = [EV() for _ in range(4)]
            with torch.cuda.stream(s):
                e[0].record(s)
                if do_h2d:
                    assert hip.hipMemcpyAsync(d_bytes.data_ptr() + b0, m_bytes.h.value + b0, b1 - b0, 1, s.cuda_stream) == 0
                    assert hip.hipMemcpyAsync(d_off.data_ptr() + 8 * lo, m_off.h.value + 8 * lo, 8 * (hi + 1 - lo), 1,
                                              s.cuda_stream) == 0
                e[1].record(s)
                if do_kernel:
                    reqs_p = (m_reqs.d.value if zero_copy else d_reqs.data_ptr()) + RS * lo
                    hdrs_p = (m_hdrs.d.value if zero_copy else d_hdrs.data_ptr()) + hbase[k]
                    b = rhp.Batch(d_bytes.data_ptr(), d_bytes.data_ptr(), d_off.data_ptr() + 8 * lo, d_bytes.numel(),
                                  hi - lo, maxh, mode, layout, reqs_p, hdrs_p,
                                  d_http.data_ptr() + (rhp.HTTP_DTYPE.itemsize * lo if mode == rhp.MODE_HTTP else 0),
                                  works[k % len(streams)].data_ptr())
                    rc = lib.rhp_parse_batch(ctypes.byref(b), ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0, rc
                e[2].record(s)
                if do_d2h and not zero_copy:
                    h_reqs[RS * lo:RS * hi].copy_(d_reqs[RS * lo:RS * hi], non_blocking=True)
                e[3].record(s)
            marks.append(e)
        rows_marks, d2h_bytes = [], RS * n if do_d2h else 0
        # header rows, on the rows stream: chunk 0's once its request records are on the
        # host; chunk k+1's speculatively, as many rows as chunks 0..k used, queued behind
        # its request records (an event wait) when chunk k's are read, so no host round
        # trip sits between the last kernel and its rows; a chunk that uses more rows than
        # guessed gets the rest when its records are read
        guess, spec = 0, {}

        def rows_copy(k, r0, r1):
            lo, hi = bounds[k], bounds[k + 1]
            a, b = hbase[k] + r0 * (hi - lo) * HB, hbase[k] + r1 * (hi - lo) * HB
            e = [EV(), EV()]
            rows_stream.wait_event(marks[k][3])   # the chunk's kernel has run (its request records copied)
            with torch.cuda.stream(rows_stream):
                e[0].record(rows_stream)
                h_hdrs[a:b].copy_(d_hdrs[a:b], non_blocking=True)
                e[1].record(rows_stream)
            rows_marks.append(e)
            return b - a

        for k in range(args.chunks):
            lo, hi = bounds[k], bounds[k + 1]
            if not do_d2h or zero_copy:   # zero copy: the kernel wrote the records into host memory
                continue
            marks[k][3].synchronize()   # chunk k's request records are on the host
            r = reqs_view[lo:hi]
            used = int(r["num_headers"][r["ret"] > 0].max(initial=0))
            have = spec.get(k, 0)
            if used > have:
                d2h_bytes += rows_copy(k, have, used)
            guess = max(guess, used)
            if k + 1 < args.chunks and guess:
                spec[k + 1] = guess
                d2h_bytes += rows_copy(k + 1, 0, guess)
            # compact: requests the exact path parsed keep their records in the chunk's wide area
            if layout == rhp.LAYOUT_COMPACT and bool((r["flags"] & rhp.F_WIDE).any()):
                w0 = hbase[k] + ((4 * (hi - lo) * maxh + 15) & ~15)
                wn = (hi - lo) * maxh * rhp.HDR_DTYPE.itemsize
                with torch.cuda.stream(rows_stream):
                    h_hdrs[w0:w0 + wn].copy_(d_hdrs[w0:w0 + wn], non_blocking=True)
                d2h_bytes += wn
        torch.cuda.synchronize()
        if timeline is not None:   # read by the caller after its clock stops
            timeline.update(t0=t0, marks=marks, rows_marks=rows_marks)
        return d2h_bytes

    def timeline_of(ev):
        ms = lambda e: ev["t0"].elapsed_time(e)   # noqa: E731
        marks, rows_marks = ev["marks"], ev["rows_marks"]
        return dict(h2d=[(ms(e[0]), ms(e[1])) for e in marks], kernel=[(ms(e[1]), ms(e[2])) for e in marks],
                    d2h_reqs=[(ms(e[2]), ms(e[3])) for e in marks], d2h_rows=[(ms(e[0]), ms(e[1])) for e in rows_marks])

    def timed(**kw):
        run(**kw)
        best, best_tl, nbytes = None, None, 0
        for _ in range(args.reps):
            ev = {}
            gc.collect()
            gc.disable()   # a collection inside the enqueue loop leaves the copy engine idle
            try:
                t0 = time.perf_counter()
                nbytes = run(timeline=ev, **kw)
                t = time.perf_counter() - t0
            finally:
                gc.enable()
            if best is None or t < best:
                best, best_tl = t, timeline_of(ev)
        return best, best_tl, nbytes

    t_e2e, tl, d2h_bytes = timed()
    reqs = reqs_view
    if zero_copy:   # the bytes the kernels wrote over PCIe: request records and used header records
        d2h_bytes = RS * n + HB * int(reqs["num_headers"][reqs["ret"] > 0].sum())
    ok_frac = float((reqs["ret"] > 0).mean())
    # what came back to the host, against the reference's digest of the same workload
    from bench import golden_spec
    spec = golden_spec(args.config, 0, n)
    parity = "unpinned: no reference digest for this size"
    if spec is not None:
        hv = np.zeros((n, maxh), dtype=rhp.HDR_DTYPE)
        raw = h_hdrs.numpy()
        for k in range(args.chunks):
            lo, hi = bounds[k], bounds[k + 1]
            hv[lo:hi] = rhp.expand_records(reqs[lo:hi], raw[hbase[k]:hbase[k + 1]], hi - lo, maxh, layout)
        res = rhp.Result(reqs.copy(), hv, None)
        parity = "match" if rhp.record_digest(*rhp.canonical(res, mode)) == spec["records_sha256"] else \
            "MISMATCH: the records copied back differ from the reference digest"
    t_h2d, _, _ = timed(do_kernel=False, do_d2h=False)
    t_kern, _, _ = timed(do_h2d=False, do_d2h=False)
    in_bytes = buf.size + off.nbytes
    gib = 2 ** 30
    busy = {k: round(_union_ms(v), 3) for k, v in tl.items()}
    span = max(b for v in tl.values() for _, b in v) if tl else 0.0
    h2d = sorted(tl.get("h2d", []))
    # where the span goes besides H2D: before the first copy, idle gaps between copies, after the last one
    h2d_edges = {"before_first_h2d_ms": round(h2d[0][0], 3) if h2d else 0.0,
                 "h2d_idle_gaps_ms": round(sum(max(0.0, b[0] - a[1]) for a, b in zip(h2d, h2d[1:])), 3),
                 "after_last_h2d_ms": round(span - h2d[-1][1], 3) if h2d else 0.0}
    result = ({
        "config": args.config, "requests": n, "algorithmic_bytes": int(alg), "chunks": args.chunks,
        "streams": args.streams, "ok_fraction": ok_frac,
        "record_layout": ("compact" if layout == rhp.LAYOUT_COMPACT else "header-major") + " per chunk",
        "records": ("written by the kernels into mapped pinned host memory (no D2H copy)" if args.records == "host"
                    else "copied back by D2H copies"),
        "parity": parity,
        "numa": numa, "taper": args.taper, "chunk_requests": [bounds[k + 1] - bounds[k] for k in range(args.chunks)],
        "e2e_GiBps": round(alg / t_e2e / gib, 2), "e2e_ms": round(t_e2e * 1e3, 3),
        "kernels_only_GiBps": round(alg / t_kern / gib, 2), "kernels_only_ms": round(t_kern * 1e3, 3),
        "h2d_GBps": round(in_bytes / t_h2d / 1e9, 2), "h2d_ms": round(t_h2d * 1e3, 3),
        "h2d_bytes": int(in_bytes), "d2h_bytes": int(d2h_bytes),
        "d2h_bytes_per_request": round(d2h_bytes / n, 2),
        # the fastest e2e repetition from HIP events: busy time (union of intervals) per engine, and the span
        "timeline_busy_ms": busy, "timeline_span_ms": round(span, 3), "timeline_h2d_edges": h2d_edges,
        "timeline_note": "h2d = bytes + offsets per chunk, kernel = rhp_parse_batch per chunk, d2h_reqs = request "
                         "records, d2h_rows = the header rows the chunk's requests use (chunk 0's issued when its "
                         "request records have landed; chunk k+1's speculatively, as many as chunks 0..k used, "
                         "behind its request records when chunk k's are read; more rows on a miss)",
    })
    del h_bytes, h_off
    m_bytes.free()
    m_off.free()
    if zero_copy:
        del h_reqs, h_hdrs, reqs_view, reqs
        m_reqs.free()
        m_hdrs.free()
    return result


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="get256", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--chunks", type=int, default=16)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--taper", type=int, default=0)
    ap.add_argument("--records", default="host", choices=["host", "copy"])
    a = ap.parse_args()
    print(json.dumps(e2e(a.config, a.n, a.chunks, a.streams, a.reps, a.taper, a.records)))


if __name__ == "__main__":
    main()
