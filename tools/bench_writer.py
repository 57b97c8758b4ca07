#!/usr/bin/env python3
"""Throughput of the batched response writer (rhp_write_responses, rhp_writer.hip):
http_write_response (src/reactor/http.c:286-297) for a batch resident in HBM.

Prints one JSON line per workload: responses/s, output GB/s (the algorithmic bytes:
every response byte is written once; body bytes are also read once) and the time
of each of the three kernels from HIP events on the launch stream.
usage: python tools/bench_writer.py [--n N] [--reps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libreactorng_amd as rhp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    for kind, n in (("plaintext", a.n), ("mixed", a.n // 8)):
        arena, resps, fields = rhp.make_responses(n, 1, kind)
        d = rhp.DeviceResponses(arena, resps, fields)
        for _ in range(3):
            d.launch()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            d.launch()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        out, off = d.result()
        total = int(off[-1])
        body = int(resps[:, 5].astype("uint64").sum())
        print(json.dumps({"workload": f"{kind}: {n} responses", "ms_per_batch": round(ms, 4),
                          "responses_per_s": round(n / ms * 1e3), "out_bytes": total,
                          "out_GBps": round(total / ms / 1e6, 1), "body_bytes_read": body,
                          "hbm_GBps_rw": round((total + body) / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
