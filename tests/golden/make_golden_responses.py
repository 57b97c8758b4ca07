#!/usr/bin/env python3
"""Generate tests/golden/responses.json from the REAL reference (dev container only).

http_write_response (src/reactor/http.c:286-297), compiled from /root/reference into
oracle/_ref/libref.so by oracle/Makefile and driven by oracle/ref_harness.c
(ref_write_responses), over deterministic response batches from
libreactorng_amd.make_responses.  Stored per set: generator parameters, sha256 of the
generated arena/records (so a GPU box regenerates identical inputs without the
reference) and sha256 of the reference's output bytes and offsets.  The three
test/http.c:143-181 cases are stored with their expected bytes as the reference test
spells them.

usage: python tests/golden/make_golden_responses.py
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
from oracle_util import reference_write_responses  # noqa: E402

SETS = [("plaintext", 4096, 1), ("mixed", 2000, 7), ("mixed", 2000, 0x5EED0006)]


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def http_c_cases():
    """test/http.c:143-181: (status, date, type, body, fields) -> expected bytes or size"""
    d = rhp.DEFAULT_DATE.decode()
    head = "HTTP/1.1 200 OK\r\nServer: *\r\nDate: " + d + "\r\nContent-Type: text/plain\r\n"
    return [
        {"status": "200 OK", "type": "text/plain", "body_hex": b"Hello".hex(), "fields": [],
         "expect": head + "Content-Length: 5\r\n\r\nHello"},
        {"status": "200 OK", "type": "text/plain", "body_hex": b"Hello, again".hex(), "fields": [["Cookie", "Test"]],
         "expect": head + "Content-Length: 12\r\nCookie: Test\r\n\r\nHello, again"},
        {"status": "200 OK", "type": "text/plain", "body_hex": bytes(1024).hex(), "fields": [], "expect_size": 1139},
    ]


def main():
    out = {"source": "oracle/_ref/libref.so: http_write_response of /root/reference/src/reactor/http.c",
           "date": rhp.DEFAULT_DATE.decode(), "sets": [], "http_c": http_c_cases()}
    for kind, n, seed in SETS:
        arena, resps, fields = rhp.make_responses(n, seed, kind)
        got, off = reference_write_responses(arena, resps, fields)
        out["sets"].append({"kind": kind, "n": n, "seed": seed, "input_sha256": sha(arena, resps, fields),
                            "out_len": int(off[-1]), "out_sha256": sha(got), "offsets_sha256": sha(off)})
        print(kind, n, seed, int(off[-1]))
    json.dump(out, open(os.path.join(HERE, "responses.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
