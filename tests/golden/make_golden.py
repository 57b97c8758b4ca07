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

Full-size BASELINE configs (1M requests; config 4 as 8 shards of 1M) are too
large to store: full_digests.json keeps the sha256 of the reference's canonical
record stream for each, which the GPU tests recompute from the kernel's output.

usage: python tests/golden/make_golden.py [--no-full] [--only NAME ...]
  --only: (re)make just the named sets of SETS / FULL, keeping every other
          fixture and manifest entry as it is
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import ctypes  # noqa: E402

import libreactorng_amd as rhp  # noqa: E402
from batches import BUILDERS, pack  # noqa: E402
from golden_sets import record_digest  # noqa: E402
from oracle_util import ORC_HDR, ORC_REQ, reference, run_reference, to_rhp  # noqa: E402

# (name, generator config, n, seed, max_headers, mode)
SETS = [
    ("tfb128_phr", rhp.GEN_TFB128, 16, 1, 16, rhp.MODE_PHR),
    ("tfb128_http", rhp.GEN_TFB128, 16, 1, 16, rhp.MODE_HTTP),
    ("get256_phr", rhp.GEN_GET256, 512, 0x5EED0002, 16, rhp.MODE_PHR),
    ("zipf_phr_h32", rhp.GEN_ZIPF, 1024, 0x5EED0003, 32, rhp.MODE_PHR),
    ("zipf_phr_h16", rhp.GEN_ZIPF, 1024, 0x5EED0003, 16, rhp.MODE_PHR),
    ("post1k_http", rhp.GEN_POST1K, 1024, 0x5EED0005, 16, rhp.MODE_HTTP),
    ("chunked_http_h16", rhp.GEN_CHUNKED, 2048, 0x5EED0006, 16, rhp.MODE_HTTP),
    ("fuzz_phr_h16", rhp.GEN_FUZZ, 4000, 11, 16, rhp.MODE_PHR),
    ("fuzz_phr_h2", rhp.GEN_FUZZ, 1500, 13, 2, rhp.MODE_PHR),
    ("fuzz_phr_h0", rhp.GEN_FUZZ, 1500, 14, 0, rhp.MODE_PHR),
    ("fuzz_http_h16", rhp.GEN_FUZZ_HTTP, 4000, 12, 16, rhp.MODE_HTTP),
    ("fuzz_http_h4", rhp.GEN_FUZZ_HTTP, 1500, 15, 4, rhp.MODE_HTTP),
]

# hand-built batches (tests/batches.py): (name, builder, align_shift, max_headers, mode)
BUILT = [
    ("long_phr_h16", "long_batch", 0, 16, rhp.MODE_PHR),
    ("long_http_h16", "long_batch", 3, 16, rhp.MODE_HTTP),
    ("long_http_h4", "long_batch", 1, 4, rhp.MODE_HTTP),
    ("edge_http_h16", "edge", 2, 16, rhp.MODE_HTTP),
    ("dense_phr_h8", "dense", 1, 8, rhp.MODE_PHR),
]

# full-size BASELINE configs: digests of the reference's canonical record stream
# (name, generator config, lo, n, seed, max_headers, mode); config 4 = config 2's
# generator at N = 8M, one digest per shard of the 8-GPU split
FULL = [
    ("config2_get256_h16", rhp.GEN_GET256, 0, 1 << 20, 0x5EED0002, 16, rhp.MODE_PHR),
    ("config3_zipf_h32", rhp.GEN_ZIPF, 0, 1 << 20, 0x5EED0003, 32, rhp.MODE_PHR),
    ("config3_zipf_h16", rhp.GEN_ZIPF, 0, 1 << 20, 0x5EED0003, 16, rhp.MODE_PHR),
    ("config5_post1k_http_h16", rhp.GEN_POST1K, 0, 1 << 20, 0x5EED0005, 16, rhp.MODE_HTTP),
    ("chunked_post_http_h16", rhp.GEN_CHUNKED, 0, 1 << 20, 0x5EED0006, 16, rhp.MODE_HTTP),
] + [(f"config4_get256_shard{g}of8", rhp.GEN_GET256, g << 20, 1 << 20, 0x5EED0002, 16, rhp.MODE_PHR)
     for g in range(8)]


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


def save_set(manifest, name, buf, off, maxh, mode, spec):
    digest = hashlib.sha256(buf.tobytes()).hexdigest()
    reqs, hdrs, http, out = run_reference(buf, off, maxh, mode)
    r, h, x = to_rhp(reqs, hdrs, http, mode)
    arrays = {"reqs": r, "hdrs": h}
    if x is not None:
        arrays["http"] = x
        arrays["bytes_out_sha256"] = np.frombuffer(hashlib.sha256(out.tobytes()).digest(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    manifest[name] = dict(spec, max_headers=maxh, mode=mode, input_sha256=digest,
                          ret_ok=int((r["ret"] > 0).sum()), ret_bad=int((r["ret"] == -1).sum()),
                          ret_partial=int((r["ret"] == -2).sum()))
    print(name, manifest[name]["ret_ok"], manifest[name]["ret_bad"], manifest[name]["ret_partial"])


def last_len_set():
    """phr_parse_request with last_len != 0 (is_complete first, picohttpparser.c:
    197-223, 399-401) over fuzz requests with seeded last_len in [0, len]."""
    buf, off = rhp.generate(rhp.GEN_FUZZ, 3000, 31)
    n = len(off) - 1
    lens = (off[1:] - off[:-1]).astype(np.int64)
    rng = np.random.default_rng(31)
    last = np.where(rng.random(n) < 0.25, 0, (rng.random(n) * (lens + 1)).astype(np.int64)).astype(np.uint64)
    ref = reference()
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    ref.ref_phr_batch_last.argtypes = [vp, vp, vp, u32, u32, vp, vp]
    reqs = np.zeros(n, dtype=ORC_REQ)
    hdrs = np.zeros((n, 16), dtype=ORC_HDR)
    ref.ref_phr_batch_last(buf.ctypes.data, off.ctypes.data, last.ctypes.data, n, 16, reqs.ctypes.data,
                           hdrs.ctypes.data)
    r, h, _ = to_rhp(reqs, hdrs, None, rhp.MODE_PHR)
    np.savez_compressed(os.path.join(HERE, "phr_last_len.npz"), reqs=r, hdrs=h, last_len=last)
    print("phr_last_len", int((r["ret"] > 0).sum()), int((r["ret"] == -1).sum()), int((r["ret"] == -2).sum()))
    return {"config": rhp.GEN_FUZZ, "n": 3000, "seed": 31, "max_headers": 16,
            "input_sha256": hashlib.sha256(buf.tobytes()).hexdigest()}


def full_digests(only=None):
    path = os.path.join(HERE, "full_digests.json")
    out = json.load(open(path))["sets"] if only else {}
    for name, cfg, lo, n, seed, maxh, mode in FULL:
        if only and name not in only:
            continue
        buf, off = rhp.generate(cfg, n, seed, lo=lo)
        reqs, hdrs, http, rw = run_reference(buf, off, maxh, mode)
        r, h, x = to_rhp(reqs, hdrs, http, mode)
        out[name] = {"config": cfg, "lo": lo, "n": n, "seed": seed, "max_headers": maxh, "mode": mode,
                     "input_sha256": hashlib.sha256(buf.tobytes()).hexdigest(),
                     "records_sha256": record_digest(r, h, x), "ret_ok": int((r["ret"] > 0).sum())}
        if cfg == rhp.GEN_CHUNKED:   # http_dechunk rewrites the bodies in place: their bytes are output too
            out[name]["bytes_out_sha256"] = hashlib.sha256(rw.tobytes()).hexdigest()
        print(name, out[name]["records_sha256"][:16], out[name]["ret_ok"])
    json.dump({"producer": "oracle/_ref/libref.so via oracle/ref_harness.c (the reference compiled from "
               "/root/reference)", "digest": "tests/golden_sets.py record_digest over to_rhp records",
               "sets": out}, open(path, "w"), indent=1)


def main_only(only):
    mpath = os.path.join(HERE, "manifest.json")
    m = json.load(open(mpath))
    for name, cfg, n, seed, maxh, mode in SETS:
        if name in only:
            buf, off = rhp.generate(cfg, n, seed)
            save_set(m["sets"], name, buf, off, maxh, mode, {"config": cfg, "n": n, "seed": seed})
    json.dump(m, open(mpath, "w"), indent=1)
    if any(name in only for name, *_ in FULL):
        full_digests(only)


def main():
    if "--only" in sys.argv:
        return main_only(set(sys.argv[sys.argv.index("--only") + 1:]))
    check_vectors()
    manifest = {}
    for name, builder, shift, maxh, mode in BUILT:
        buf, off = pack(BUILDERS[builder](), align_shift=shift)
        save_set(manifest, name, buf, off, maxh, mode, {"builder": builder, "align_shift": shift, "n": len(off) - 1})
    for name, cfg, n, seed, maxh, mode in SETS:
        buf, off = rhp.generate(cfg, n, seed)
        save_set(manifest, name, buf, off, maxh, mode, {"config": cfg, "n": n, "seed": seed})
    last = last_len_set()
    json.dump({"generator": "include/rhp_gen.h (splitmix64); builder sets: tests/batches.py",
               "producer": "oracle/_ref/libref.so via oracle/ref_harness.c (the reference compiled from "
               "/root/reference)", "sets": manifest, "phr_last_len": last},
              open(os.path.join(HERE, "manifest.json"), "w"), indent=1)
    if "--no-full" not in sys.argv:
        full_digests()


if __name__ == "__main__":
    main()
