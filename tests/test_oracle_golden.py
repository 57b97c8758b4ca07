"""CPU: the oracle, the DFA emulator and the product's CPU exact parser against
golden fixtures produced by the REAL reference (tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import libreactorng_amd as rhp
from golden_sets import inputs, record_digest
from oracle_util import assert_same, canon, run_oracle, to_rhp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
SETS = MANIFEST["sets"]
FULL = json.load(open(os.path.join(GOLDEN, "full_digests.json")))["sets"]


def load_golden(name):
    spec = SETS[name]
    buf, off = inputs(spec)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    want = (z["reqs"], z["hdrs"], z["http"] if "http" in z.files else None)
    return spec, buf, off, want, z


@pytest.mark.parametrize("name", sorted(SETS))
def test_oracle_matches_reference_golden(name):
    spec, buf, off, want, z = load_golden(name)
    reqs, hdrs, http, out = run_oracle(buf, off, spec["max_headers"], spec["mode"])
    got = to_rhp(reqs, hdrs, http, spec["mode"])
    assert_same(got, want, buf, off, f"oracle vs reference golden {name}")
    if "bytes_out_sha256" in z.files:
        assert hashlib.sha256(out.tobytes()).digest() == z["bytes_out_sha256"].tobytes()


@pytest.mark.parametrize("layout", [rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_HEADER_MAJOR, rhp.LAYOUT_COMPACT])
@pytest.mark.parametrize("name", sorted(SETS))
def test_dfa_emulation_matches_golden(name, layout):
    spec, buf, off, want, z = load_golden(name)
    res, stats = rhp.emulate(buf, off, spec["max_headers"], spec["mode"], layout)
    assert_same(canon(res, spec["mode"]), want, buf, off, f"DFA emulation vs golden {name}")
    if layout == rhp.LAYOUT_COMPACT and spec["mode"] == rhp.MODE_HTTP:
        # compact http records (rhp.h rhp_http_compact_t): the DFA-framed requests are stored
        # compact, only the exact path's and de-framed chunked bodies' records are wide
        flags = res.raw_http[:8 * len(res.reqs)].reshape(-1, 8)[:, 2]
        wide = (flags & 1) != 0
        dfa = (res.reqs["flags"] & 1) == 0
        assert wide[~dfa].all(), "exact-path records are wide"
        if name.startswith("config5"):   # Content-Length POSTs: framed in the DFA path
            assert (~wide[dfa]).mean() > 0.9, "DFA-framed records are compact"
    if "bytes_out_sha256" in z.files:
        assert hashlib.sha256(res.bytes_out.tobytes()).digest() == z["bytes_out_sha256"].tobytes()


@pytest.mark.parametrize("name", sorted(SETS))
def test_cpu_exact_parser_matches_golden(name):
    spec, buf, off, want, z = load_golden(name)
    res = rhp.parse_cpu_exact(buf, off, spec["max_headers"], spec["mode"], rhp.LAYOUT_HEADER_MAJOR)
    assert_same(canon(res, spec["mode"]), want, buf, off, f"CPU exact parser vs golden {name}")
    # compact layout (phr and, ADVICE r5, http records): every record wide (RHP_F_WIDE), expanded the same
    res = rhp.parse_cpu_exact(buf, off, spec["max_headers"], spec["mode"], rhp.LAYOUT_COMPACT)
    assert_same(canon(res, spec["mode"]), want, buf, off, f"CPU exact parser (compact) vs golden {name}")
    assert ((res.reqs["flags"] & rhp.F_WIDE) != 0).all()
    if spec["mode"] == rhp.MODE_HTTP:
        hc = res.raw_http[: 8 * (len(off) - 1)].view(np.uint8).reshape(-1, 8)
        assert (hc[:, 2] & rhp.HTTP_WIDE).all(), "every compact http record of the exact path is wide"


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


def test_pointer_parser_last_len_matches_reference_golden():
    """rhp_phr_parse_request (phr_parse_request's signature, pointer outputs) with
    last_len != 0 -- is_complete first (picohttpparser.c:197-223, 399-401) --
    against the compiled reference's answers (tests/golden/phr_last_len.npz)."""
    spec = MANIFEST["phr_last_len"]
    buf, off = inputs(spec)
    z = np.load(os.path.join(GOLDEN, "phr_last_len.npz"))
    for i in range(len(off) - 1):
        ret, minor, m, p, hs = rhp.phr_parse_request_cpu(buf, int(off[i]), int(off[i + 1] - off[i]), 16,
                                                         int(z["last_len"][i]))
        w = z["reqs"][i]
        assert ret == w["ret"], (i, ret, w)
        if ret > 0:
            assert (minor, m, p) == (w["minor_version"], (w["method_off"], w["method_len"]),
                                     (w["path_off"], w["path_len"])), i
            want = [(-1 if h["name_off"] == rhp.RHP_NAME_NULL else int(h["name_off"]), int(h["name_len"]),
                     int(h["value_off"]), int(h["value_len"])) for h in z["hdrs"][i][: int(w["num_headers"])]]
            assert hs == want, i


@pytest.mark.parametrize("name", ["config2_get256_h16", "config5_post1k_http_h16", "config4_get256_shard7of8",
                                  "chunked_post_http_h16"])
def test_oracle_full_size_matches_reference_digest(name):
    """The restatement at BASELINE full size (1M requests) against the digest of
    the compiled reference's record stream (tests/golden/full_digests.json), and
    of the de-chunked bytes where http_dechunk rewrote them."""
    spec = FULL[name]
    buf, off = inputs(spec)
    reqs, hdrs, http, out = run_oracle(buf, off, spec["max_headers"], spec["mode"])
    got = to_rhp(reqs, hdrs, http, spec["mode"])
    assert record_digest(*got) == spec["records_sha256"]
    if "bytes_out_sha256" in spec:
        assert hashlib.sha256(out.tobytes()).hexdigest() == spec["bytes_out_sha256"]


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="needs the reference sources (dev container)")
def test_diff_fuzz_oracle_vs_compiled_reference():
    """A short run of oracle/diff_fuzz.c: the restatement against the reference
    compiled from /root/reference (every generator config x max_headers, phr
    and http mode, rewritten bytes included).  The long runs (>= 10^7 requests)
    are logged under profiles/ by tools/run_diff_fuzz.sh."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "oracle"), "ref"])
    out = subprocess.run([os.path.join(root, "oracle", "_ref", "diff_fuzz"), "42", "2000", "7"], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0 and "diff_fuzz OK: 84000 requests" in out.stdout, out.stdout + out.stderr


@pytest.mark.parametrize("layout", [rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_HEADER_MAJOR])
def test_batch_last_len_emulation_matches_reference_golden(layout):
    """rhp_batch_t.last_len (phr mode): the kernel's decisions (rhp_emu.cpp) with
    is_complete first where last_len != 0 (picohttpparser.c:197-223, 399-401),
    against the compiled reference's answers (tests/golden/phr_last_len.npz)."""
    spec = MANIFEST["phr_last_len"]
    buf, off = inputs(spec)
    z = np.load(os.path.join(GOLDEN, "phr_last_len.npz"))
    res, stats = rhp.emulate(buf, off, 16, rhp.MODE_PHR, layout, last_len=z["last_len"])
    assert_same(canon(res, rhp.MODE_PHR), (z["reqs"], z["hdrs"], None), buf, off, "emulation, last_len")
    assert stats[0] > 0   # the DFA path still answers the requests is_complete cannot change


def last_len_sweep():
    """Each request of a mixed set repeated with last_len = 0 .. len + 3 (the
    contract's range), in one batch."""
    b1, o1 = rhp.generate(rhp.GEN_FUZZ, 120, 77)
    b2, o2 = rhp.generate(rhp.GEN_GET256, 4, 78)
    reqs = [bytes(b1[o1[i]:o1[i + 1]]) for i in range(len(o1) - 1)]
    reqs += [bytes(b2[o2[i]:o2[i + 1]]) for i in range(len(o2) - 1)]
    rep, last = [], []
    for r in reqs:
        for ll in sorted(set(list(range(0, min(len(r), 12) + 4)) + list(range(max(0, len(r) - 8), len(r) + 4)))):
            rep.append(r)
            last.append(ll)
    from batches import pack
    buf, off = pack(rep)
    return buf, off, np.array(last, dtype=np.uint64)


def test_batch_last_len_sweep_emulation_vs_pointer_parser():
    buf, off, last = last_len_sweep()
    res, _ = rhp.emulate(buf, off, 16, rhp.MODE_PHR, last_len=last)
    for i in range(len(off) - 1):
        ret, minor, m, p, hs = rhp.phr_parse_request_cpu(buf, int(off[i]), int(off[i + 1] - off[i]), 16, int(last[i]))
        r = res.reqs[i]
        assert r["ret"] == ret, (i, int(last[i]), r, ret)
        if ret > 0:
            assert (r["minor_version"], (r["method_off"], r["method_len"]), (r["path_off"], r["path_len"])) == \
                (minor, m, p), i
            got = [(-1 if h["name_off"] == rhp.RHP_NAME_NULL else int(h["name_off"]), int(h["name_len"]),
                    int(h["value_off"]), int(h["value_len"])) for h in res.hdrs[i][: int(r["num_headers"])]]
            assert got == hs, i
