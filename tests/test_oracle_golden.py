"""CPU: the oracle, the DFA emulator and the product's CPU exact parser against
golden fixtures produced by the REAL reference (tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import libreactorng_amd as rhp
from oracle_util import assert_same, canon, run_oracle, to_rhp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))["sets"]


def load_golden(name):
    spec = MANIFEST[name]
    buf, off = rhp.generate(spec["config"], spec["n"], spec["seed"])
    assert hashlib.sha256(buf.tobytes()).hexdigest() == spec["input_sha256"], "generator drifted"
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    want = (z["reqs"], z["hdrs"], z["http"] if "http" in z.files else None)
    return spec, buf, off, want, z


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_oracle_matches_reference_golden(name):
    spec, buf, off, want, z = load_golden(name)
    reqs, hdrs, http, out = run_oracle(buf, off, spec["max_headers"], spec["mode"])
    got = to_rhp(reqs, hdrs, http, spec["mode"])
    assert_same(got, want, buf, off, f"oracle vs reference golden {name}")
    if "bytes_out_sha256" in z.files:
        assert hashlib.sha256(out.tobytes()).digest() == z["bytes_out_sha256"].tobytes()


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_dfa_emulation_matches_golden(name):
    spec, buf, off, want, z = load_golden(name)
    res, stats = rhp.emulate(buf, off, spec["max_headers"], spec["mode"])
    assert_same(canon(res, spec["mode"]), want, buf, off, f"DFA emulation vs golden {name}")
    if "bytes_out_sha256" in z.files:
        assert hashlib.sha256(res.bytes_out.tobytes()).digest() == z["bytes_out_sha256"].tobytes()


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_cpu_exact_parser_matches_golden(name):
    spec, buf, off, want, z = load_golden(name)
    res = rhp.parse_cpu_exact(buf, off, spec["max_headers"], spec["mode"])
    assert_same(canon(res, spec["mode"]), want, buf, off, f"CPU exact parser vs golden {name}")


def vectors():
    return json.load(open(os.path.join(GOLDEN, "http_request_tests.json")))


def one_request(s: bytes):
    off = np.array([0, len(s)], dtype=np.uint64)
    buf = np.zeros(len(s) + rhp.RHP_PAD, dtype=np.uint8)
    buf[: len(s)] = np.frombuffer(s, dtype=np.uint8)
    return buf, off


@pytest.mark.parametrize("i", range(21))
def test_reference_http_vectors(i):
    """test/http.c:121-141: result and remaining bytes after http_read_request."""
    spec = vectors()
    v = spec["vectors"][i]
    buf, off = one_request(v["request"].encode("latin-1"))
    L = int(off[1])
    for run in ("oracle", "emulation", "cpu_exact"):
        if run == "oracle":
            _, _, http, _ = run_oracle(buf, off, 16, rhp.MODE_HTTP)
            result, consumed = int(http["result"][0]), int(http["consumed"][0])
        else:
            res = (rhp.emulate(buf, off, 16, rhp.MODE_HTTP)[0] if run == "emulation"
                   else rhp.parse_cpu_exact(buf, off, 16, rhp.MODE_HTTP))
            result, consumed = int(res.http["result"][0]), int(res.http["consumed"][0])
        remaining = L - consumed if result == 1 else L
        assert (result, remaining) == (v["result"], v["remaining"]), (run, v)


def test_known_answer_tfb128():
    """SURVEY.md §8c KAT: ret=128 method=(0,3) path=(4,10) minor=1, 4 headers."""
    buf, off = rhp.generate(rhp.GEN_TFB128, 1, 1)
    reqs, hdrs, http, _ = run_oracle(buf, off, 16)
    r, h, _ = to_rhp(reqs, hdrs, http, rhp.MODE_PHR)
    assert r["ret"][0] == 128 and r["method_off"][0] == 0 and r["method_len"][0] == 3
    assert r["path_off"][0] == 4 and r["path_len"][0] == 10 and r["minor_version"][0] == 1
    assert r["num_headers"][0] == 4
    assert [tuple(int(x) for x in h[0][k]) for k in range(4)] == [
        (25, 4, 31, 15), (48, 6, 56, 10), (68, 10, 80, 10), (92, 10, 104, 20)]
    res, _ = rhp.emulate(buf, off, 16)
    assert_same(canon(res, rhp.MODE_PHR), (r, h, None), buf, off, "KAT emulation")
