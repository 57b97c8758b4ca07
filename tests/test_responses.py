"""Batched response serialization: http_write_response (src/reactor/http.c:286-297).

CPU: the oracle restatement (oracle/rhp_oracle.c orc_write_responses) against the
golden digests the real reference produced (tests/golden/responses.json,
make_golden_responses.py) and against the test/http.c:143-181 cases; against the
compiled reference itself when /root/reference is present.
GPU: rhp_write_responses (rhp_writer.hip) byte-exact against the oracle.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import libreactorng_amd as rhp
from oracle_util import oracle_write_responses, reference, reference_write_responses

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "responses.json")))


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def http_c_batch():
    """the test/http.c:143-181 cases as one batch"""
    parts, resps, fields = [], [], []
    pos = 0

    def add(b: bytes):
        nonlocal pos
        parts.append(b)
        pos += len(b)
        return [pos - len(b), len(b)]

    for c in GOLDEN["http_c"]:
        st, ty, body = add(c["status"].encode()), add(c["type"].encode()), add(bytes.fromhex(c["body_hex"]))
        first = len(fields)
        for name, value in c["fields"]:
            fields.append(add(name.encode()) + add(value.encode()))
        resps.append(st + ty + body + [first, len(c["fields"])])
    arena = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return arena, np.array(resps, dtype=np.uint32), np.array(fields, dtype=np.uint32).reshape(-1, 4)


def check_http_c(out, off):
    for i, c in enumerate(GOLDEN["http_c"]):
        got = bytes(out[int(off[i]):int(off[i + 1])])
        if "expect" in c:
            assert got == c["expect"].encode(), (i, got)
        else:
            assert len(got) == c["expect_size"], (i, len(got))


@pytest.mark.parametrize("s", GOLDEN["sets"], ids=lambda s: f"{s['kind']}-{s['seed']}")
def test_oracle_matches_reference_golden(s):
    arena, resps, fields = rhp.make_responses(s["n"], s["seed"], s["kind"])
    assert sha(arena, resps, fields) == s["input_sha256"], "generator drifted from the golden inputs"
    out, off = oracle_write_responses(arena, resps, fields)
    assert int(off[-1]) == s["out_len"]
    assert sha(off) == s["offsets_sha256"]
    assert sha(out) == s["out_sha256"]


def test_oracle_http_c_vectors():
    check_http_c(*oracle_write_responses(*http_c_batch()))


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs /root/reference (dev container)")
def test_oracle_matches_reference_fresh_seeds():
    assert reference() is not None
    for seed in (101, 102):
        a, r, f = rhp.make_responses(700, seed, "mixed")
        o1, f1 = oracle_write_responses(a, r, f)
        o2, f2 = reference_write_responses(a, r, f)
        assert np.array_equal(f1, f2) and np.array_equal(o1, o2)
    check_http_c(*reference_write_responses(*http_c_batch()))


def test_writer_argument_errors():
    """C-ABI checks that need no GPU: NULL batch, wrong date length"""
    import ctypes
    lib = rhp.lib()
    assert lib.rhp_write_responses(None, None) == -22
    b = rhp.RespBatch(None, None, None, 0, 28, b"x" * 28, 8, None, 0)
    assert lib.rhp_write_responses(ctypes.byref(b), None) == -22


# ------------------------------------------------------------------ GPU


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,seed", [("plaintext", 4096, 1), ("mixed", 2000, 7), ("mixed", 5000, 99),
                                         ("mixed", 1, 3)])
def test_gpu_writer_matches_oracle(kind, n, seed):
    arena, resps, fields = rhp.make_responses(n, seed, kind)
    got, off = rhp.write_responses(arena, resps, fields)
    want, woff = oracle_write_responses(arena, resps, fields)
    assert np.array_equal(off, woff)
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_writer_golden_and_http_c():
    for s in GOLDEN["sets"]:
        arena, resps, fields = rhp.make_responses(s["n"], s["seed"], s["kind"])
        got, off = rhp.write_responses(arena, resps, fields)
        assert sha(off) == s["offsets_sha256"] and sha(got) == s["out_sha256"], s
    check_http_c(*rhp.write_responses(*http_c_batch()))


@pytest.mark.gpu
def test_gpu_writer_edges():
    # empty batch: out_off[0] = 0, nothing else touched
    d = rhp.DeviceResponses(np.zeros(1, np.uint8), np.zeros((0, 8), np.uint32), np.zeros((0, 4), np.uint32))
    d.launch()
    out, off = d.result()
    assert len(off) == 1 and off[0] == 0 and len(out) == 0
    # too small an output: the offsets are complete, the output untouched
    arena, resps, fields = rhp.make_responses(300, 5, "mixed")
    d = rhp.DeviceResponses(arena, resps, fields, out_size=1000)
    d.launch()
    _, off = d.result()
    _, woff = oracle_write_responses(arena, resps, fields)
    assert np.array_equal(off, woff)
    assert int(d.out.cpu().numpy().astype(np.int64).sum()) == 0


@pytest.mark.gpu
def test_gpu_writer_plaintext_1m():
    """1M TechEmpower plaintext replies: every response is the same 126 bytes"""
    arena, resps, fields = rhp.make_responses(1 << 20, 1, "plaintext")
    got, off = rhp.write_responses(arena, resps, fields)
    one, _ = oracle_write_responses(arena, resps[:1], fields)
    assert len(got) == len(one) << 20
    assert np.array_equal(got.reshape(1 << 20, len(one)), np.broadcast_to(one, (1 << 20, len(one))))
    assert np.array_equal(off, np.arange((1 << 20) + 1, dtype=np.uint64) * len(one))
