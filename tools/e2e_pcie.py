"""End-to-end rate from host memory to host memory (north_star: "this path starts and
ends in host memory -- the io_uring recv buffer").

The batch (config 2 by default: 1M x 256 B) sits in pinned host memory; it is cut
into chunks that stream through S HIP streams: pinned hipMemcpyAsync H2D of the
chunk's bytes and offsets -> rhp_parse_batch on that chunk -> D2H of its request
records and header records.  Copies of one chunk overlap the kernel of another
and the two copy directions overlap each other.  Reports GiB/s of algorithmic
bytes over the wall time of the whole batch, next to the device-resident kernel
rate of the same batch and the copy-only rates.

usage: python tools/e2e_pcie.py [--config get256] [--chunks 16] [--streams 3] [--reps 5]
"""
import argparse
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


def e2e(config="get256", n=1 << 20, chunks=16, streams=3, reps=5):
    """The end-to-end measurement as a dict (bench.py's `e2e` object)."""
    args = argparse.Namespace(config=config, n=n, chunks=chunks, streams=streams, reps=reps)
    cfg = CONFIGS[args.config]
    n, maxh, mode = args.n, cfg["maxh"], cfg["mode"]
    buf, off = rhp.generate(cfg["gen"], n, cfg["seed"])
    alg = rhp.header_bytes(cfg["gen"], n, cfg["seed"])
    dev = torch.device("cuda")

    # pinned host buffers (the recv side) and full-size device mirrors
    h_bytes = torch.from_numpy(buf).pin_memory()
    h_off = torch.from_numpy(off.view(np.int64)).pin_memory()
    h_reqs = torch.empty(n * rhp.REQ_DTYPE.itemsize, dtype=torch.uint8).pin_memory()
    h_hdrs = torch.empty(n * maxh * rhp.HDR_DTYPE.itemsize, dtype=torch.uint8).pin_memory()
    d_bytes = torch.empty_like(h_bytes, device=dev)
    d_off = torch.empty_like(h_off, device=dev)
    d_reqs = torch.empty_like(h_reqs, device=dev)
    d_hdrs = torch.empty_like(h_hdrs, device=dev)
    d_http = torch.zeros(max(1, n if mode == rhp.MODE_HTTP else 1) * rhp.HTTP_DTYPE.itemsize,
                         dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream() for _ in range(args.streams)]
    works = [torch.zeros(rhp.RHP_WORK_WORDS, dtype=torch.int32, device=dev) for _ in streams]
    lib = rhp.lib()
    bounds = [n * k // args.chunks for k in range(args.chunks + 1)]
    RS, HS = rhp.REQ_DTYPE.itemsize, maxh * rhp.HDR_DTYPE.itemsize

    def run(do_h2d=True, do_kernel=True, do_d2h=True):
        for k in range(args.chunks):
            lo, hi = bounds[k], bounds[k + 1]
            s = streams[k % len(streams)]
            b0, b1 = int(off[lo]), int(off[hi]) + rhp.RHP_PAD   # the chunk's bytes + the pad the ABI reads
            b1 = min(b1, buf.size)
            with torch.cuda.stream(s):
                if do_h2d:
                    d_bytes[b0:b1].copy_(h_bytes[b0:b1], non_blocking=True)
                    d_off[lo:hi + 1].copy_(h_off[lo:hi + 1], non_blocking=True)
                if do_kernel:
                    b = rhp.Batch(d_bytes.data_ptr(), d_bytes.data_ptr(), d_off.data_ptr() + 8 * lo, d_bytes.numel(),
                                  hi - lo, maxh, mode, 0, d_reqs.data_ptr() + RS * lo, d_hdrs.data_ptr() + HS * lo,
                                  d_http.data_ptr() + (rhp.HTTP_DTYPE.itemsize * lo if mode == rhp.MODE_HTTP else 0),
                                  works[k % len(streams)].data_ptr())
                    rc = lib.rhp_parse_batch(ctypes.byref(b), ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0, rc
                if do_d2h:
                    h_reqs[RS * lo:RS * hi].copy_(d_reqs[RS * lo:RS * hi], non_blocking=True)
                    h_hdrs[HS * lo:HS * hi].copy_(d_hdrs[HS * lo:HS * hi], non_blocking=True)
        torch.cuda.synchronize()

    def timed(**kw):
        run(**kw)
        t = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            run(**kw)
            t.append(time.perf_counter() - t0)
        return min(t)

    t_e2e = timed()
    # parity of what came back to the host: the template answer for config 2
    reqs = h_reqs.numpy().view(rhp.REQ_DTYPE)
    ok_frac = float((reqs["ret"] > 0).mean())
    t_h2d = timed(do_kernel=False, do_d2h=False)
    t_d2h = timed(do_h2d=False, do_kernel=False)
    t_kern = timed(do_h2d=False, do_d2h=False)
    in_bytes = buf.size + off.nbytes
    out_bytes = h_reqs.numel() + h_hdrs.numel()
    gib = 2 ** 30
    return ({
        "config": args.config, "requests": n, "algorithmic_bytes": int(alg), "chunks": args.chunks,
        "streams": args.streams, "ok_fraction": ok_frac,
        "e2e_GiBps": round(alg / t_e2e / gib, 2), "e2e_ms": round(t_e2e * 1e3, 3),
        "kernels_only_GiBps": round(alg / t_kern / gib, 2), "kernels_only_ms": round(t_kern * 1e3, 3),
        "h2d_GBps": round(in_bytes / t_h2d / 1e9, 2), "h2d_ms": round(t_h2d * 1e3, 3),
        "d2h_GBps": round(out_bytes / t_d2h / 1e9, 2), "d2h_ms": round(t_d2h * 1e3, 3),
        "h2d_bytes": int(in_bytes), "d2h_bytes": int(out_bytes),
    })


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="get256", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--chunks", type=int, default=16)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    print(json.dumps(e2e(a.config, a.n, a.chunks, a.streams, a.reps)))


if __name__ == "__main__":
    main()
