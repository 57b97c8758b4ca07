"""CPU: generator determinism and sharding, library exports, DFA emulation fuzz
against the oracle, edge cases of the batch contract."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import libreactorng_amd as rhp
from batches import EDGE, dense_header_batch, long_batch, pack  # noqa: F401
from oracle_util import assert_same, canon, run_oracle, to_rhp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rhp_[a-z_0-9]+)\s*\(", text, re.M)))


def exported(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_librhp_exports_every_declared_symbol():
    decl = declared_functions("rhp.h")
    assert set(decl) == set(rhp.RHP_SYMBOLS), decl
    have = exported(rhp.LIBRHP)
    missing = [s for s in decl if s not in have]
    assert not missing, missing
    lib = rhp.lib()           # loads without a GPU; no compute call here
    assert lib.rhp_version().startswith(b"rhp")
    assert lib.rhp_set_impl(7) == -22 and lib.rhp_set_impl(0) == 0


def test_host_lib_exports():
    decl = declared_functions("rhp_gen.h")
    have = exported(rhp.LIBHOST)
    assert not [s for s in decl if s not in have]
    for s in rhp.HOST_SYMBOLS:
        assert s in have, s


def test_parse_batch_argument_errors_without_gpu():
    lib = rhp.lib()
    assert lib.rhp_parse_batch(None, None) == -22
    b = rhp.Batch()
    assert lib.rhp_parse_batch(ctypes.byref(b), None) == 0        # n == 0: nothing to do
    b.n = 5
    assert lib.rhp_parse_batch(ctypes.byref(b), None) == -22      # null pointers rejected
    b.n, b.bytes, b.offsets, b.reqs, b.work, b.hdrs = 5, 17, 8, 8, 8, 8
    assert lib.rhp_parse_batch(ctypes.byref(b), None) == -22      # bytes not 16-byte aligned
    b.bytes = 16
    b.max_headers = rhp.RHP_MAX_HEADERS + 1
    assert lib.rhp_parse_batch(ctypes.byref(b), None) == -22      # capacity limit
    b.max_headers, b.mode = 16, 7
    assert lib.rhp_parse_batch(ctypes.byref(b), None) == -22      # unknown mode


@pytest.mark.parametrize("cfg", [1, 2, 3, 5, 100, 101])
def test_generator_deterministic_and_shardable(cfg):
    a, oa = rhp.generate(cfg, 300, 42)
    b, ob = rhp.generate(cfg, 300, 42)
    assert np.array_equal(a, b) and np.array_equal(oa, ob)
    assert np.all(a[int(oa[-1]):] == 0) and len(a) - int(oa[-1]) == rhp.RHP_PAD
    s, os_ = rhp.generate(cfg, 100, 42, lo=120)
    assert bytes(s[: int(os_[-1])]) == bytes(a[int(oa[120]):int(oa[220])])
    assert np.array_equal(os_, oa[120:221] - oa[120])


def test_config_shapes():
    buf, off = rhp.generate(rhp.GEN_GET256, 64, 0x5EED0002)
    assert np.all(np.diff(off) == 256)
    buf, off = rhp.generate(rhp.GEN_POST1K, 2000, 0x5EED0005)
    assert np.all(np.diff(off) == 1024)
    hb = rhp.header_bytes(rhp.GEN_POST1K, 2000, 0x5EED0005)
    assert 2000 * 128 < hb < 2000 * 170
    buf, off = rhp.generate(rhp.GEN_ZIPF, 20000, 0x5EED0003)
    lens = np.diff(off)
    assert lens.min() >= 18 and lens.max() <= 4096
    assert 500 < lens.mean() < 800   # mean ~642 B


@pytest.mark.parametrize("seed", [101, 202, 303])
@pytest.mark.parametrize("maxh", [0, 1, 5, 16, 64])
def test_dfa_emulation_fuzz_vs_oracle(seed, maxh):
    for cfg, mode in ((rhp.GEN_FUZZ, rhp.MODE_PHR), (rhp.GEN_FUZZ_HTTP, rhp.MODE_HTTP)):
        buf, off = rhp.generate(cfg, 6000, seed + maxh)
        res, stats = rhp.emulate(buf, off, maxh, mode)
        want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
        assert_same(canon(res, mode), want, buf, off, f"emu cfg{cfg} seed{seed} maxh{maxh}")
        if mode == rhp.MODE_PHR:   # compact records: the running sum of rhp.h gives the same offsets
            res, _ = rhp.emulate(buf, off, maxh, mode, rhp.LAYOUT_COMPACT)
            assert_same(canon(res, mode), want, buf, off, f"emu compact seed{seed} maxh{maxh}")


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
@pytest.mark.parametrize("maxh", [0, 1, 16])
def test_edge_cases_emulation(shift, maxh):
    buf, off = pack(EDGE, align_shift=shift)
    for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
        res, _ = rhp.emulate(buf, off, maxh, mode)
        want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
        assert_same(canon(res, mode), want, buf, off, f"edge shift{shift} maxh{maxh} mode{mode}")


def test_max_headers_boundary():
    """17 headers with capacity 16 -> -1; exactly 16 -> ok."""
    def req(k):
        return b"GET / HTTP/1.1\r\n" + b"".join(b"H%d: v\r\n" % i for i in range(k)) + b"\r\n"
    buf, off = pack([req(15), req(16), req(17), req(40)])
    res, _ = rhp.emulate(buf, off, 16)
    assert list(res.reqs["ret"][:2] > 0) == [True, True] and list(res.reqs["ret"][2:]) == [-1, -1]
    want = to_rhp(*run_oracle(buf, off, 16)[:3], rhp.MODE_PHR)
    assert_same(canon(res, rhp.MODE_PHR), want, buf, off, "max headers")


def test_toolong_request_reported():
    """A header section longer than the u16 records (ret > 65535) is the one
    answer the batch format cannot carry: RHP_RET_TOOLONG (include/rhp.h)."""
    big = b"GET /" + b"a" * 70000 + b" HTTP/1.1\r\n\r\n"
    buf, off = pack([b"GET / HTTP/1.1\r\n\r\n", big])
    res, _ = rhp.emulate(buf, off, 16)
    assert res.reqs["ret"][0] == 18 and res.reqs["ret"][1] == rhp.RHP_RET_TOOLONG
    # the pointer-based host parser has no such limit
    assert rhp.phr_parse_request_cpu(buf, int(off[1]), len(big), 16)[0] == len(big)


@pytest.mark.parametrize("maxh", [4, 16, 64])
def test_long_inputs_emulation_and_host_vs_oracle(maxh):
    buf, off = pack(long_batch())
    for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
        want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
        res, _ = rhp.emulate(buf, off, maxh, mode)
        assert_same(canon(res, mode), want, buf, off, f"long inputs emulation maxh{maxh} mode{mode}")
        res = rhp.parse_cpu_exact(buf, off, maxh, mode)
        assert_same(canon(res, mode), want, buf, off, f"long inputs host exact maxh{maxh} mode{mode}")


def test_long_inputs_pointer_parser_vs_oracle():
    """rhp_phr_parse_request / rhp_http_read_cpu (pointer outputs, no limit)
    against the oracle's wide records, including header sections > 64 KiB."""
    buf, off = pack(long_batch())
    for maxh in (4, 16):
        reqs, hdrs, _, _ = run_oracle(buf, off, maxh, rhp.MODE_PHR)
        for i in range(len(off) - 1):
            got = rhp.phr_parse_request_cpu(buf, int(off[i]), int(off[i + 1] - off[i]), maxh)
            r = reqs[i]
            assert got[0] == r["ret"], (i, got[0], r)
            if r["ret"] > 0:
                assert got[1] == r["minor_version"]
                assert got[2] == (r["method_off"], r["method_len"]) and got[3] == (r["path_off"], r["path_len"])
                want_h = [tuple(int(v) for v in hdrs[i, k]) for k in range(int(r["num_headers"]))]
                assert got[4] == want_h, i
        rw = buf.copy()
        _, _, http, _ = run_oracle(buf, off, maxh, rhp.MODE_HTTP)
        for i in range(len(off) - 1):
            res, consumed, body = rhp.http_read_cpu(rw, int(off[i]), int(off[i + 1] - off[i]), maxh)
            assert res == http["result"][i], (i, res, http[i])
            if res == 1:
                assert consumed == http["consumed"][i]
                assert (body is not None) == bool(http["body_kind"][i])


@pytest.mark.parametrize("shift", [0, 3])
def test_dense_headers_emulation(shift):
    buf, off = pack(dense_header_batch(), align_shift=shift)
    for maxh in (0, 6, 7, 8, 16, 64):
        for mode in (rhp.MODE_PHR, rhp.MODE_HTTP):
            res, _ = rhp.emulate(buf, off, maxh, mode)
            want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
            assert_same(canon(res, mode), want, buf, off, f"dense shift{shift} maxh{maxh} mode{mode}")


@pytest.mark.parametrize("mode", [rhp.MODE_PHR, rhp.MODE_HTTP])
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_emulator_version_errors_vs_oracle(mode, shift):
    """A version that is not HTTP/1.<digit> at every cut length: the emulator of
    the kernel's algorithm (its DFA ERR with the PE + 10 length rule) against the
    oracle."""
    from batches import version_batch
    buf, off = pack(version_batch(), align_shift=shift)
    emu, _ = rhp.emulate(buf, off, 16, mode)
    want = to_rhp(*run_oracle(buf, off, 16, mode)[:3], mode)
    assert_same(canon(emu, mode), want, buf, off, f"emu version mode{mode} shift{shift}")


def test_chunk_window_equals_one_chunk_t():
    """The GPU replay's windowed size-line parse (rhp_scalar.h one_chunk_window)
    against the byte-wise one_chunk_t (http.c:73-132) on random size lines:
    wherever the window decides, the result and the data span are one_chunk_t's,
    and it decides every line whose LF lies in its 17-32 bytes (or whose body
    ends there); the bytes past the window are garbage it must not read."""
    import ctypes
    import random
    h = rhp.host()
    h.rhp_test_chunk_window.restype = ctypes.c_int
    h.rhp_test_chunk_window.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_void_p] * 3
    h.rhp_test_chunk_exact.restype = ctypes.c_int64
    alpha = b"0123456789abcdefABCDEF \t;\r\nxgz=\x00" + b"0" * 8 + b"\r\n" * 4
    rng = random.Random(5)
    res, doff, dlen = ctypes.c_int64(), ctypes.c_uint64(), ctypes.c_uint64()
    d2, l2 = ctypes.c_uint64(), ctypes.c_uint64()
    decided = 0
    for it in range(60000):
        kind = it % 4
        if kind == 0:   # well-formed: OWS? hex OWS? ext? CRLF data CRLF
            line = (b" " * rng.randrange(3) + f"{rng.randrange(1 << rng.randrange(1, 64)):x}".encode()
                    + rng.choice([b"", b"\t", b" \t"]) + rng.choice([b"", b";ext=1", b";a\rb"]) + b"\r\n")
        else:
            line = bytes(rng.choice(alpha) for _ in range(rng.randrange(0, 40)))
        body = line + bytes(rng.randrange(256) for _ in range(rng.randrange(0, 64)))
        size = rng.randrange(0, len(body) + 1) if rng.random() < 0.5 else len(body)
        buf = (ctypes.c_uint8 * (size + 128))(*body[:size])   # zeros past the body, as the padded batch
        want = h.rhp_test_chunk_exact(buf, 0, size, ctypes.byref(d2), ctypes.byref(l2))
        nw = 32 if it % 2 else rng.randrange(17, 33)   # the kernel's two lines hold 17..32 bytes from the line
        win = (ctypes.c_uint8 * 32)(*(bytes(buf)[:nw] + bytes(rng.randrange(256) for _ in range(32 - nw))))
        ok = h.rhp_test_chunk_window(win, nw, size, ctypes.byref(res), ctypes.byref(doff), ctypes.byref(dlen))
        nl = bytes(buf)[:nw].find(b"\n")
        if nl >= 0 or size <= nw:
            assert ok == 1, (line, size, nw)
        if ok:
            decided += 1
            assert res.value == want, (line, size, res.value, want)
            if want > 0:
                assert (doff.value, dlen.value) == (d2.value, l2.value), (line, size)
    assert decided > 50000


def test_chunk_head_equals_one_chunk_t():
    """The replay's branch-free size-line parse (rhp_scalar.h one_chunk_head: the
    LF by a zero-byte test, the state machine over the first 8 bytes) against the
    byte-wise one_chunk_t (http.c:73-132) and one_chunk_window, on the same kind
    of random size lines as above, for the kernel's 20-byte window (5 dwords,
    nw 17-20) and a 32-byte one: wherever it decides, the result and the data
    span are one_chunk_t's; it decides every well-formed line of this workload's
    shape (OWS, up to 8 digits or an extension within 8 bytes)."""
    import ctypes
    import random
    h = rhp.host()
    h.rhp_test_chunk_head.restype = ctypes.c_int
    h.rhp_test_chunk_head.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_void_p] * 3 + [ctypes.c_uint32]
    h.rhp_test_chunk_window.restype = ctypes.c_int
    h.rhp_test_chunk_window.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64] + [ctypes.c_void_p] * 3
    h.rhp_test_chunk_exact.restype = ctypes.c_int64
    alpha = b"0123456789abcdefABCDEF \t;\r\nxgz=\x00" + b"0" * 8 + b"\r\n" * 4
    rng = random.Random(7)
    res, doff, dlen = ctypes.c_int64(), ctypes.c_uint64(), ctypes.c_uint64()
    d2, l2 = ctypes.c_uint64(), ctypes.c_uint64()
    decided = common = 0
    for it in range(80000):
        kind = it % 4
        short = kind == 0 and it % 8 == 0   # the bench workload's shape
        if kind == 0:
            line = (b" " * rng.randrange(2 if short else 3) + f"{rng.randrange(1 << rng.randrange(1, 12 if short else 64)):x}".encode()
                    + rng.choice([b"", b"\t"] if short else [b"", b"\t", b" \t"])
                    + rng.choice([b"", b";ext=1", b";a\rb"]) + b"\r\n")
        else:
            line = bytes(rng.choice(alpha) for _ in range(rng.randrange(0, 40)))
        body = line + bytes(rng.randrange(256) for _ in range(rng.randrange(0, 64)))
        size = rng.randrange(0, len(body) + 1) if rng.random() < 0.5 else len(body)
        buf = (ctypes.c_uint8 * (size + 128))(*body[:size])
        want = h.rhp_test_chunk_exact(buf, 0, size, ctypes.byref(d2), ctypes.byref(l2))
        nd = 5 if it % 2 else 8
        nw = rng.randrange(17, 21) if nd == 5 else rng.randrange(17, 33)
        win = (ctypes.c_uint8 * 32)(*(bytes(buf)[:nw] + bytes(rng.randrange(256) for _ in range(32 - nw))))
        ok = h.rhp_test_chunk_head(win, nw, size, ctypes.byref(res), ctypes.byref(doff), ctypes.byref(dlen), nd)
        if ok:
            decided += 1
            assert res.value == want, (line, size, nw, nd, res.value, want)
            if want > 0:
                assert (doff.value, dlen.value) == (d2.value, l2.value), (line, size, nd)
        if short and size == len(body) and line.find(b";") < 0:
            common += 1
            assert ok == 1, (line, size, nw, nd)
    assert decided > 50000 and common > 1500


def test_emulator_chunked_paths_vs_oracle():
    """The GPU's chunked-paths batch (tests/batches.py chunked_paths_batch) through
    the kernel emulation: records and rewritten bytes equal the oracle's."""
    from batches import chunked_paths_batch, pack
    from oracle_util import assert_same, canon, run_oracle, to_rhp
    buf, off = pack(chunked_paths_batch(n=3000), align_shift=5)
    res, _ = rhp.emulate(buf, off, 16, rhp.MODE_HTTP)
    reqs, hdrs, http, rw = run_oracle(buf, off, 16, rhp.MODE_HTTP)
    assert_same(canon(res, rhp.MODE_HTTP), to_rhp(reqs, hdrs, http, rhp.MODE_HTTP), buf, off, "emulated chunked paths")
    assert np.array_equal(res.bytes_out, rw)
