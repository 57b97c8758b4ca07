#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REAL reference (dev container only).

The reference is compiled from /root/reference by oracle/Makefile into
oracle/_ref/libref.so (never committed); this script drives it through
oracle/ref_harness.c over deterministic batches from the in-repo generator
(include/rhp_gen.h) and stores, per fixture set:
  - the generator parameters and the sha256 of the generated input bytes
    (so the GPU box regenerates identical inputs without the reference),
  - the reference's records in the compact rhp.h layout (canonical: fields the
    reference leaves unspecified are zeroed), as a compressed .npz.
It also checks the transcribed test/http.c vectors (http_request_tests.json)
against the compiled reference.

usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import libreactorng_amd as rhp  # noqa: E402
from oracle_util import run_reference, to_rhp  # noqa: E402

# (name, generator config, n, seed, max_headers, mode)
SETS = [
    ("tfb128_phr", rhp.GEN_TFB128, 16, 1, 16, rhp.MODE_PHR),
    ("tfb128_http", rhp.GEN_TFB128, 16, 1, 16, rhp.MODE_HTTP),
    ("get256_phr", rhp.GEN_GET256, 512, 0x5EED0002, 16, rhp.MODE_PHR),
    ("zipf_phr_h32", rhp.GEN_ZIPF, 1024, 0x5EED0003, 32, rhp.MODE_PHR),
    ("zipf_phr_h16", rhp.GEN_ZIPF, 1024, 0x5EED0003, 16, rhp.MODE_PHR),
    ("post1k_http", rhp.GEN_POST1K, 1024, 0x5EED0005, 16, rhp.MODE_HTTP),
    ("fuzz_phr_h16", rhp.GEN_FUZZ, 4000, 11, 16, rhp.MODE_PHR),
    ("fuzz_phr_h2", rhp.GEN_FUZZ, 1500, 13, 2, rhp.MODE_PHR),
    ("fuzz_phr_h0", rhp.GEN_FUZZ, 1500, 14, 0, rhp.MODE_PHR),
    ("fuzz_http_h16", rhp.GEN_FUZZ_HTTP, 4000, 12, 16, rhp.MODE_HTTP),
    ("fuzz_http_h4", rhp.GEN_FUZZ_HTTP, 1500, 15, 4, rhp.MODE_HTTP),
]


def vectors_batch(vecs):
    """Pack the test/http.c vectors as one batch (each followed by the next)."""
    parts = [v["request"].encode("latin-1") for v in vecs]
    off = np.zeros(len(parts) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(p) for p in parts])
    buf = np.zeros(int(off[-1]) + rhp.RHP_PAD, dtype=np.uint8)
    buf[: int(off[-1])] = np.frombuffer(b"".join(parts), dtype=np.uint8)
    return buf, off


def check_vectors():
    spec = json.load(open(os.path.join(HERE, "http_request_tests.json")))
    vecs = spec["vectors"]
    # each vector alone (the reference test runs them one stream at a time)
    for v in vecs:
        buf, off = vectors_batch([v])
        reqs, hdrs, http, _ = run_reference(buf, off, spec["max_headers"], rhp.MODE_HTTP)
        L = int(off[1])
        remaining = L - int(http["consumed"][0]) if http["result"][0] == 1 else L
        assert int(http["result"][0]) == v["result"] and remaining == v["remaining"], (v, http[0])
    print(f"test/http.c vectors: {len(vecs)}/{len(vecs)} match the compiled reference")


def main():
    check_vectors()
    manifest = {}
    for name, cfg, n, seed, maxh, mode in SETS:
        buf, off = rhp.generate(cfg, n, seed)
        digest = hashlib.sha256(buf.tobytes()).hexdigest()
        reqs, hdrs, http, out = run_reference(buf, off, maxh, mode)
        r, h, x = to_rhp(reqs, hdrs, http, mode)
        arrays = {"reqs": r, "hdrs": h}
        if x is not None:
            arrays["http"] = x
            arrays["bytes_out_sha256"] = np.frombuffer(hashlib.sha256(out.tobytes()).digest(), dtype=np.uint8)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        manifest[name] = {"config": cfg, "n": n, "seed": seed, "max_headers": maxh, "mode": mode,
                          "input_sha256": digest,
                          "ret_ok": int((r["ret"] > 0).sum()), "ret_bad": int((r["ret"] == -1).sum()),
                          "ret_partial": int((r["ret"] == -2).sum())}
        print(name, manifest[name]["ret_ok"], manifest[name]["ret_bad"], manifest[name]["ret_partial"])
    json.dump({"generator": "include/rhp_gen.h (splitmix64)", "producer": "oracle/_ref/libref.so via "
               "oracle/ref_harness.c (the reference compiled from /root/reference)", "sets": manifest},
              open(os.path.join(HERE, "manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
