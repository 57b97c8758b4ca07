"""GPU parity: the HIP kernels (through the C-ABI in librhp.so) against the
reference's golden fixtures and the oracle, bit-exact, at fixture sizes and at
BASELINE.json full sizes."""
import hashlib
import json
import os

import numpy as np
import pytest

import libreactorng_amd as rhp
from golden_sets import inputs, record_digest
from oracle_util import assert_same, canon, run_oracle, to_rhp
from batches import EDGE, chunked_paths_batch, dense_header_batch, long_batch, pack

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))["sets"]
FULL = json.load(open(os.path.join(GOLDEN, "full_digests.json")))["sets"]


def golden(name):
    spec = MANIFEST[name]
    buf, off = inputs(spec)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    return spec, buf, off, (z["reqs"], z["hdrs"], z["http"] if "http" in z.files else None), z


@pytest.mark.parametrize("impl,layout", [(rhp.IMPL_DFA, rhp.LAYOUT_REQUEST_MAJOR), (rhp.IMPL_EXACT, rhp.LAYOUT_REQUEST_MAJOR),
                                         (rhp.IMPL_DFA, rhp.LAYOUT_HEADER_MAJOR), (rhp.IMPL_EXACT, rhp.LAYOUT_HEADER_MAJOR),
                                         (rhp.IMPL_DFA_LATE, rhp.LAYOUT_REQUEST_MAJOR),
                                         (rhp.IMPL_DFA_LATE, rhp.LAYOUT_HEADER_MAJOR),
                                         (rhp.IMPL_DFA, rhp.LAYOUT_COMPACT), (rhp.IMPL_EXACT, rhp.LAYOUT_COMPACT),
                                         (rhp.IMPL_DFA_LATE, rhp.LAYOUT_COMPACT)])
@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_gpu_matches_reference_golden(name, impl, layout):
    spec, buf, off, want, z = golden(name)
    res = rhp.parse_batch(buf, off, spec["max_headers"], spec["mode"], impl=impl, layout=layout)
    assert_same(canon(res, spec["mode"]), want, buf, off, f"GPU impl{impl} vs golden {name}")
    if "bytes_out_sha256" in z.files:
        assert hashlib.sha256(res.bytes_out.tobytes()).digest() == z["bytes_out_sha256"].tobytes()


def test_gpu_reference_http_vectors():
    spec = json.load(open(os.path.join(GOLDEN, "http_request_tests.json")))
    for v in spec["vectors"]:
        s = v["request"].encode("latin-1")
        buf, off = pack([s])
        res = rhp.parse_batch(buf, off, 16, rhp.MODE_HTTP)
        result, consumed = int(res.http["result"][0]), int(res.http["consumed"][0])
        remaining = len(s) - consumed if result == 1 else len(s)
        assert (result, remaining) == (v["result"], v["remaining"]), v


@pytest.mark.parametrize("maxh", [0, 1, 3, 16, 32, 64])
def test_gpu_compact_fuzz_vs_oracle(maxh):
    """Compact records (RHP_LAYOUT_COMPACT): lengths from the DFA, wide records
    from the exact path (RHP_F_WIDE) exactly where the emulator takes it; the
    expanded records equal the oracle's."""
    for cfg, mode, impl, seed in ((rhp.GEN_FUZZ, rhp.MODE_PHR, rhp.IMPL_DFA, 9300 + maxh),
                                  (rhp.GEN_FUZZ, rhp.MODE_PHR, rhp.IMPL_DFA_LATE, 9400 + maxh),
                                  (rhp.GEN_FUZZ_HTTP, rhp.MODE_HTTP, rhp.IMPL_DFA, 9500 + maxh)):
        buf, off = rhp.generate(cfg, 60000, seed)
        res = rhp.parse_batch(buf, off, maxh, mode, impl=impl, layout=rhp.LAYOUT_COMPACT)
        want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
        assert_same(canon(res, mode), want, buf, off, f"GPU compact fuzz cfg{cfg} impl{impl} maxh{maxh}")
        emu, _ = rhp.emulate(buf, off, maxh, mode, rhp.LAYOUT_COMPACT)
        assert np.array_equal(res.reqs["flags"] & (rhp.F_EXACT | rhp.F_WIDE), emu.reqs["flags"] & (rhp.F_EXACT | rhp.F_WIDE))
        if mode == rhp.MODE_HTTP:   # de-framed bytes too; exact-path http records are wide
            assert (res.bytes_out == run_oracle(buf, off, maxh, mode)[3]).all()
            wide = (res.raw_http[:8 * len(res.reqs)].reshape(-1, 8)[:, 2] & 1) != 0
            assert wide[(res.reqs["flags"] & rhp.F_EXACT) != 0].all()


@pytest.mark.parametrize("name", ["config2_get256_h16", "config3_zipf_h32", "config4_get256_shard5of8",
                                  "config5_post1k_http_h16", "chunked_post_http_h16"])
def test_gpu_compact_full_size_matches_reference_digest(name):
    spec = FULL[name]
    buf, off = inputs(spec)
    res = rhp.parse_batch(buf, off, spec["max_headers"], spec["mode"], layout=rhp.LAYOUT_COMPACT)
    got = canon(res, spec["mode"])
    if record_digest(*got) != spec["records_sha256"]:
        want = to_rhp(*run_oracle(buf, off, spec["max_headers"], spec["mode"])[:3], spec["mode"])
        assert_same(got, want, buf, off, name)
        raise AssertionError(f"{name}: compact digest differs from the reference but matches the oracle")
    if "bytes_out_sha256" in spec:
        assert hashlib.sha256(res.bytes_out.tobytes()).hexdigest() == spec["bytes_out_sha256"]


@pytest.mark.parametrize("maxh", [0, 1, 3, 16, 32, 64])
def test_gpu_fuzz_vs_oracle(maxh):
    for cfg, mode, seed, impl in ((rhp.GEN_FUZZ, rhp.MODE_PHR, 9000 + maxh, rhp.IMPL_DFA),
                                  (rhp.GEN_FUZZ, rhp.MODE_PHR, 9200 + maxh, rhp.IMPL_DFA_LATE),
                                  (rhp.GEN_FUZZ_HTTP, rhp.MODE_HTTP, 9100 + maxh, rhp.IMPL_DFA)):
        buf, off = rhp.generate(cfg, 60000, seed)
        res = rhp.parse_batch(buf, off, maxh, mode, impl=impl)
        want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
        assert_same(canon(res, mode), want, buf, off, f"GPU fuzz cfg{cfg} maxh{maxh}")
        # the kernel takes the exact path for exactly the requests the emulator of
        # its algorithm (rhp_emu.cpp) sends there
        emu, _ = rhp.emulate(buf, off, maxh, mode)
        assert np.array_equal(res.reqs["flags"] & rhp.F_EXACT, emu.reqs["flags"] & rhp.F_EXACT)


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_gpu_edge_cases(shift):
    buf, off = pack(EDGE * 3, align_shift=shift)
    for maxh in (0, 1, 16):
        for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
            want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
            for layout in (rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_COMPACT):
                res = rhp.parse_batch(buf, off, maxh, mode, layout=layout)
                assert_same(canon(res, mode), want, buf, off, f"GPU edge shift{shift} maxh{maxh} mode{mode} layout{layout}")


def test_gpu_toolong_and_empty_batch():
    """Only a header section longer than the u16 records (ret > 65535) is
    RHP_RET_TOOLONG; a 70 KB request whose header section is short parses."""
    big = b"GET /" + b"a" * 70000 + b" HTTP/1.1\r\n\r\n"
    long_tail = b"GET / HTTP/1.1\r\n\r\n" + b"x" * 70000
    buf, off = pack([b"GET / HTTP/1.1\r\n\r\n", big, b"", long_tail])
    for impl in (rhp.IMPL_DFA, rhp.IMPL_EXACT):
        res = rhp.parse_batch(buf, off, 16, impl=impl)
        assert list(res.reqs["ret"]) == [18, rhp.RHP_RET_TOOLONG, -2, 18]
        res = rhp.parse_batch(buf, off, 16, rhp.MODE_HTTP, impl=impl)
        assert list(res.http["result"]) == [1, rhp.RHP_RET_TOOLONG, 0, 1]
    buf, off = pack([])
    res = rhp.parse_batch(buf, off, 16)
    assert len(res.reqs) == 0


@pytest.mark.parametrize("impl", [rhp.IMPL_DFA, rhp.IMPL_EXACT])
@pytest.mark.parametrize("shift", [0, 1, 3])
def test_gpu_long_inputs_vs_oracle(impl, shift):
    """Inputs past 64 KiB (200 KB / 1 MiB Content-Length POSTs, ~70 KiB of
    pipelined GETs, chunked bodies, errors and partials past 64 KiB) bit-exact
    vs the oracle, bytes rewritten in place included."""
    buf, off = pack(long_batch(), align_shift=shift)
    for maxh in (4, 16):
        for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
            res = rhp.parse_batch(buf, off, maxh, mode, impl=impl)
            reqs, hdrs, http, rw = run_oracle(buf, off, maxh, mode)
            assert_same(canon(res, mode), to_rhp(reqs, hdrs, http, mode), buf, off,
                        f"GPU long inputs impl{impl} shift{shift} maxh{maxh} mode{mode}")
            if mode == rhp.MODE_HTTP:
                assert np.array_equal(res.bytes_out, rw)


@pytest.mark.parametrize("shift,n", [(0, 6000), (5, 6000), (12, 6000), (3, 160000)])
def test_gpu_chunked_paths_vs_oracle(shift, n):
    """Every de-framing path of the replay (staged groups, tiny chunks, many
    chunks, bodies beyond a slot, long size lines, bodies ending at the request's
    end, malformed and partial framing), records and rewritten bytes bit-exact
    vs the oracle (http.c:73-160); a neighbour's bytes are never written.  At
    160K requests a workgroup defers more than its list holds: the second pass
    then takes the range itself (no first pass)."""
    buf, off = pack(chunked_paths_batch(n), align_shift=shift)
    res = rhp.parse_batch(buf, off, 16, rhp.MODE_HTTP)
    reqs, hdrs, http, rw = run_oracle(buf, off, 16, rhp.MODE_HTTP)
    assert_same(canon(res, rhp.MODE_HTTP), to_rhp(reqs, hdrs, http, rhp.MODE_HTTP), buf, off, f"chunked paths shift{shift}")
    assert np.array_equal(res.bytes_out, rw), f"{int((res.bytes_out != rw).sum())} rewritten bytes differ"
    assert (http["body_kind"] == 1).sum() > n // 2


def test_gpu_repeated_launches_rearm_work_counter():
    buf, off = rhp.generate(rhp.GEN_ZIPF, 5000, 77)
    db = rhp.DeviceBatch(buf, off, 32)
    want = to_rhp(*run_oracle(buf, off, 32)[:3], rhp.MODE_PHR)
    for _ in range(5):
        db.reqs.zero_()
        db.launch()
        assert_same(canon(db.result(), rhp.MODE_PHR), want, buf, off, "relaunch")


def test_gpu_full_size_config2_properties():
    """BASELINE config 2 at full size (1M x 256 B): every record equals the template
    answer shifted by the 138 B path; a 64K slice compared against the oracle."""
    n = 1 << 20
    buf, off = rhp.generate(rhp.GEN_GET256, n, 0x5EED0002)
    res = rhp.parse_batch(buf, off, 16)
    r = res.reqs
    assert np.all(r["ret"] == 256) and np.all(r["path_off"] == 4) and np.all(r["path_len"] == 138)
    assert np.all(r["method_len"] == 3) and np.all(r["minor_version"] == 1) and np.all(r["num_headers"] == 4)
    assert np.all(r["flags"] == 0)
    h = res.hdrs[:, :4]
    kat = [(25, 4, 31, 15), (48, 6, 56, 10), (68, 10, 80, 10), (92, 10, 104, 20)]
    for k, (no, nl, vo, vl) in enumerate(kat):
        assert np.all(h[:, k]["name_off"] == no + 128) and np.all(h[:, k]["name_len"] == nl)
        assert np.all(h[:, k]["value_off"] == vo + 128) and np.all(h[:, k]["value_len"] == vl)
    lo, hi = n - 65536, n
    s, so = rhp.generate(rhp.GEN_GET256, hi - lo, 0x5EED0002, lo=lo)
    want = to_rhp(*run_oracle(s, so, 16)[:3], rhp.MODE_PHR)
    got = canon(rhp.Result(r[lo:hi], res.hdrs[lo:hi], None), rhp.MODE_PHR)
    assert_same(got, want, s, so, "config 2 tail slice")


@pytest.mark.parametrize("cfg,maxh,mode", [(rhp.GEN_ZIPF, 32, rhp.MODE_PHR), (rhp.GEN_ZIPF, 16, rhp.MODE_PHR),
                                           (rhp.GEN_POST1K, 16, rhp.MODE_HTTP)])
def test_gpu_full_size_configs_vs_oracle(cfg, maxh, mode):
    """BASELINE configs 3 and 5 at full size (1M requests), bit-exact vs the oracle."""
    n = 1 << 20
    seed = {rhp.GEN_ZIPF: 0x5EED0003, rhp.GEN_POST1K: 0x5EED0005}[cfg]
    buf, off = rhp.generate(cfg, n, seed)
    res = rhp.parse_batch(buf, off, maxh, mode)
    want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
    assert_same(canon(res, mode), want, buf, off, f"full size cfg{cfg} maxh{maxh}")


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_gpu_dense_headers(shift):
    buf, off = pack(dense_header_batch(4000, 11 + shift), align_shift=shift)
    for maxh in (0, 6, 7, 8, 16, 64):
        for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
            res = rhp.parse_batch(buf, off, maxh, mode)
            want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
            assert_same(canon(res, mode), want, buf, off, f"GPU dense shift{shift} maxh{maxh} mode{mode}")


@pytest.mark.parametrize("name", sorted(FULL))
def test_gpu_full_size_matches_reference_digest(name):
    """BASELINE configs 2, 3 (max_headers 32 and 16), 5 at full size and every
    shard of config 4 (8M requests over 8 GPUs, shard g = requests [g*2^20,
    (g+1)*2^20)): the kernel's canonical record stream hashes to the digest of
    the compiled reference's (tests/golden/full_digests.json)."""
    spec = FULL[name]
    buf, off = inputs(spec)
    layout = rhp.LAYOUT_HEADER_MAJOR if "shard" in name else rhp.LAYOUT_REQUEST_MAJOR
    res = rhp.parse_batch(buf, off, spec["max_headers"], spec["mode"], layout=layout)
    got = canon(res, spec["mode"])
    if record_digest(*got) != spec["records_sha256"]:   # say which request differs
        want = to_rhp(*run_oracle(buf, off, spec["max_headers"], spec["mode"])[:3], spec["mode"])
        assert_same(got, want, buf, off, name)
        raise AssertionError(f"{name}: digest differs from the reference but matches the oracle")
    if "bytes_out_sha256" in spec:   # chunked bodies de-framed in place (http.c:134-160)
        if hashlib.sha256(res.bytes_out.tobytes()).hexdigest() != spec["bytes_out_sha256"]:
            out = run_oracle(buf, off, spec["max_headers"], spec["mode"])[3]
            bad = np.nonzero(out != res.bytes_out)[0]
            raise AssertionError(f"{name}: {len(bad)} rewritten bytes differ, first at {bad[:8]}")


@pytest.mark.parametrize("impl", [rhp.IMPL_DFA, rhp.IMPL_DFA_LATE])
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_gpu_version_errors(impl, shift):
    """Versions that are not HTTP/1.<digit>, cut at every length (batches.version_batch):
    -1 from the DFA only when the version's 9 bytes are there, else the exact path."""
    from batches import version_batch
    buf, off = pack(version_batch() * 2, align_shift=shift)
    for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
        res = rhp.parse_batch(buf, off, 16, mode, impl=impl)
        want = to_rhp(*run_oracle(buf, off, 16, mode)[:3], mode)
        assert_same(canon(res, mode), want, buf, off, f"GPU version impl{impl} shift{shift} mode{mode}")


@pytest.mark.parametrize("impl,layout", [(rhp.IMPL_DFA, rhp.LAYOUT_REQUEST_MAJOR), (rhp.IMPL_DFA, rhp.LAYOUT_HEADER_MAJOR),
                                         (rhp.IMPL_DFA_LATE, rhp.LAYOUT_REQUEST_MAJOR),
                                         (rhp.IMPL_EXACT, rhp.LAYOUT_REQUEST_MAJOR)])
def test_gpu_last_len_matches_reference_golden(impl, layout):
    """rhp_batch_t.last_len: is_complete first where last_len != 0
    (picohttpparser.c:197-223, 399-401), against the reference's answers."""
    top = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    buf, off = inputs(top["phr_last_len"])
    z = np.load(os.path.join(GOLDEN, "phr_last_len.npz"))
    res = rhp.parse_batch(buf, off, 16, rhp.MODE_PHR, impl=impl, layout=layout, last_len=z["last_len"])
    assert_same(canon(res, rhp.MODE_PHR), (z["reqs"], z["hdrs"], None), buf, off, f"GPU impl{impl} last_len")


def test_gpu_last_len_sweep_vs_emulation():
    """Every last_len in 0 .. len + 3 on fuzz and config-2 requests: the GPU
    equals the kernel emulation (itself pinned to the pointer parser on CPU)."""
    from test_oracle_golden import last_len_sweep
    buf, off, last = last_len_sweep()
    want, _ = rhp.emulate(buf, off, 16, rhp.MODE_PHR, last_len=last)
    for impl in (rhp.IMPL_DFA, rhp.IMPL_EXACT):
        res = rhp.parse_batch(buf, off, 16, rhp.MODE_PHR, impl=impl, last_len=last)
        assert_same(canon(res, rhp.MODE_PHR), canon(want, rhp.MODE_PHR), buf, off, f"GPU impl{impl} last_len sweep")


@pytest.mark.parametrize("mode", [rhp.MODE_PHR, rhp.MODE_HTTP])
def test_gpu_batch_over_4gib(mode):
    """A batch larger than 4 GiB: a first request of 4 GiB + 4 KiB (its
    workgroup's range cannot use the u32 window offsets and runs the exact path)
    and 300k config-2 requests behind it, at absolute offsets above 4 GiB, on
    the DFA path.  Expected records: the oracle on the same requests packed
    without the giant one (a request's records depend only on its own bytes and
    the bytes after it)."""
    head = b"GET /big HTTP/1.1\r\nHost: x\r\n\r\n"
    big = (1 << 32) + 4096 + 3
    nb, no = rhp.generate(rhp.GEN_GET256, 300000, 4242)
    nbytes = int(no[-1])
    buf = np.zeros(big + nbytes + rhp.RHP_PAD, dtype=np.uint8)
    buf[:len(head)] = np.frombuffer(head, dtype=np.uint8)
    buf[big:big + nbytes] = nb[:nbytes]
    off = np.concatenate([np.zeros(1, dtype=np.uint64), no.astype(np.uint64) + np.uint64(big)])
    res = rhp.parse_batch(buf, off, 16, mode)
    got = canon(res, mode)
    want = to_rhp(*run_oracle(nb, no, 16, mode)[:3], mode)
    assert_same(tuple(x[1:] if x is not None else None for x in got), want, nb, no, "over 4 GiB: the requests after")
    sbuf, soff = pack([head + bytes(64)])
    w0 = to_rhp(*run_oracle(sbuf, soff, 16, mode)[:3], mode)
    assert got[0][0] == w0[0][0] and (got[1][0] == w0[1][0]).all()
    if mode == rhp.MODE_HTTP:
        assert got[2][0] == w0[2][0]
    del res, buf
