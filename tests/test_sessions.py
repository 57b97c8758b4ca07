"""Pipelined input in one batch: every session's input is
split at its empty lines, the pieces are parsed as one speculative batch, and
rhp_fixup_sessions walks each session in order.  The result must equal the
reference's server_session_read loop (server.c:37-65): http_read_request
(http.c:177-234) from the front of the input, advancing by what it consumed,
until it returns 0 or -1 -- here the oracle restatement called per request at
the true boundaries of the same batch buffer (so the bytes after a session are
the same in both), de-framing chunked bodies in place as the reference does.

Streams mix GETs, Content-Length bodies (some holding empty lines and whole
fake requests), chunked bodies (also with empty lines inside), LF-only line
ends, malformed requests and incomplete tails.  CPU: the product's exact host
parser and the kernel's DFA emulation; GPU (-m gpu): the MI355X kernels."""
import ctypes

import numpy as np
import pytest

import libreactorng_amd as rhp
from oracle_util import ORC_HDR, ORC_HTTP, ORC_REQ, oracle

TFB = (b"GET /plaintext HTTP/1.1\r\nHost: tfb-server:8080\r\nAccept: text/plain\r\n"
       b"Connection: keep-alive\r\nUser-Agent: wrk/4.2.0 (tfb-load)\r\n\r\n")


def request_pool(rng):
    fake = b"GET /inside-a-body HTTP/1.1\r\nHost: x\r\n\r\n"
    body = b"line one\r\n\r\n" + fake + b"\n\ntail"
    chunk_data = b"ab\r\n\r\ncd"
    pool = [
        TFB,
        b"GET / HTTP/1.1\r\nHost: a\r\n\r\n",
        b"GET /lf HTTP/1.1\nX: y\n\n",
        b"GET /mix HTTP/1.0\r\nA: b\n\r\n",
        b"POST /cl HTTP/1.1\r\nContent-Length: 5\r\n\r\nhello",
        b"POST /cl-empty-lines HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % len(body) + body,
        b"POST /c HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n",
        b"POST /c2 HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n%x\r\n" % len(chunk_data) + chunk_data +
        b"\r\n0\r\n\r\n",
        b"PUT /zero HTTP/1.1\r\nContent-Length: 0\r\n\r\n",
        b"GET /h HTTP/1.1\r\n" + b"".join(b"H%d: v\r\n" % i for i in range(16)) + b"\r\n",
    ]
    bad = [b"GET /x HTTP/1.1\r\nBad Header\r\n\r\n", b"POST /b HTTP/1.1\r\nContent-Length: 3\r\n"
           b"Transfer-Encoding: chunked\r\n\r\nabc", b"GET / HTTP/2.0\r\n\r\n",
           b"POST /c HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n"]
    tails = [b"GET /last HTTP/1.1\r\nHost:", b"POST /p HTTP/1.1\r\nContent-Length: 100\r\n\r\nonly-part",
             b"POST /c HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhel", b""]
    return pool, bad, tails


def make_sessions(n_sessions, seed):
    rng = np.random.default_rng(seed)
    pool, bad, tails = request_pool(rng)
    out = []
    for _ in range(n_sessions):
        k = int(rng.integers(1, 40))
        parts = [pool[int(rng.integers(len(pool)))] for _ in range(k)]
        if rng.random() < 0.1:
            parts.insert(int(rng.integers(len(parts) + 1)), bad[int(rng.integers(len(bad)))])
        parts.append(tails[int(rng.integers(len(tails)))])
        out.append(b"".join(parts))
    return out


def oracle_sessions(buf, off, sessions, max_headers=16):
    """Per session: [(result, start, consumed, method, path, fields, body)] of the
    reference's loop, and the batch bytes after it (chunked bodies de-framed)."""
    o = oracle()
    rw = buf.copy()
    reqs = np.zeros(1, dtype=ORC_REQ)
    hdrs = np.zeros((1, max_headers), dtype=ORC_HDR)
    http = np.zeros(1, dtype=ORC_HTTP)
    one = np.zeros(2, dtype=np.uint64)
    out = []
    for lo, hi in sessions:
        pos, end, seq = int(off[lo]), int(off[hi]), []
        while pos < end:
            one[0], one[1] = pos, end
            o.orc_http_batch(rw.ctypes.data, one.ctypes.data, 1, max_headers, reqs.ctypes.data, hdrs.ctypes.data,
                             http.ctypes.data)
            res = int(http["result"][0])
            r = reqs[0]
            if res == 1 and r["ret"] > rhp.RHP_MAX_LEN:
                res = rhp.RHP_RET_TOOLONG
            if res != 1:
                seq.append((res, pos, 0, None, None, None, None))
                break
            b = bytes(rw[pos:end])
            fields = [(b"" if h["name_off"] < 0 else b[h["name_off"]:h["name_off"] + h["name_len"]],
                       b[h["value_off"]:h["value_off"] + h["value_len"]]) for h in hdrs[0][: int(r["num_headers"])]]
            body = b""
            if http["body_kind"][0]:
                bo = int(http["body_off"][0])
                body = b[bo:bo + int(http["body_len"][0])]
            c = int(http["consumed"][0])
            seq.append((1, pos, c, b[r["method_off"]:r["method_off"] + r["method_len"]],
                        b[r["path_off"]:r["path_off"] + r["path_len"]], fields, body))
            pos += c
        out.append(seq)
    return out, rw


def product_sessions(res, results, starts, off, sessions, allow_more=False):
    """The same view of rhp_fixup_sessions' output."""
    out = []
    rw = res.bytes_out
    for (lo, hi), sr in zip(sessions, results):
        end, seq = int(off[hi]), []
        for m in range(int(sr["n_slots"])):
            i = lo + m
            x, r, pos = res.http[i], res.reqs[i], int(starts[i])
            if x["result"] != 1:
                seq.append((int(x["result"]), pos, 0, None, None, None, None))
                break
            b = bytes(rw[pos:end])
            fields = [(b"" if h["name_off"] == rhp.RHP_NAME_NULL else b[h["name_off"]:h["name_off"] + h["name_len"]],
                       b[h["value_off"]:h["value_off"] + h["value_len"]]) for h in res.hdrs[i][: int(r["num_headers"])]]
            body = b[int(r["ret"]):int(r["ret"]) + int(x["body_len"])] if x["body_kind"] else b""
            seq.append((1, pos, int(x["consumed"]), b[r["method_off"]:r["method_off"] + r["method_len"]],
                        b[r["path_off"]:r["path_off"] + r["path_len"]], fields, body))
        assert allow_more or not sr["more"]
        out.append(seq)
    return out


def check(res, results, starts, buf, off, sess, label, allow_more=False):
    sessions = [(int(a), int(b)) for a, b in sess]
    want, want_bytes = oracle_sessions(buf, off, sessions)
    got = product_sessions(res, results, starts, off, sessions, allow_more)
    if allow_more:   # a session that ran out of pieces: its first n_slots requests, the rest in a later batch
        want = [w[: len(g)] if sr["more"] else w for g, w, sr in zip(got, want, results)]
        want_bytes = None
    for k, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"{label}: session {k}: first difference at request " \
                       f"{next(i for i in range(min(len(g), len(w)) + 1) if i >= min(len(g), len(w)) or g[i] != w[i])}"
    n = int(off[-1])
    if want_bytes is not None:
        assert bytes(res.bytes_out[:n]) == bytes(want_bytes[:n]), f"{label}: de-framed bytes differ"
    return sum(len(w) for w in want)


def test_split_pieces():
    assert rhp.split_pieces(b"GET / HTTP/1.1\r\n\r\nGET / HTTP/1.1\n\nX") == [18, 16, 1]
    assert rhp.split_pieces(b"") == [0]
    assert rhp.split_pieces(b"abc") == [3]
    assert rhp.split_pieces(b"A\n\r\n") == [4]


@pytest.mark.parametrize("emulate_dfa", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fixup_cpu_matches_reference_loop(seed, emulate_dfa):
    data = make_sessions(60, seed)
    buf, off, sess, _ = rhp.pack_sessions(data)
    res, results, starts = rhp.fixup_cpu(buf, off, sess, 16, emulate_dfa)
    total = check(res, results, starts, buf, off, sess, f"cpu seed {seed}")
    assert total > 60


def test_fixup_cpu_unsplit_sessions():
    """One piece per session: the first request of each is the piece's own
    speculative result (chunked bodies validated, then de-framed by the
    fix-up: RHP_BODY_CHUNKED_PENDING), the rest runs out of pieces (more)."""
    data = make_sessions(80, 9)
    buf, off, sess, _ = rhp.pack_sessions(data, split=False)
    res, results, starts = rhp.fixup_cpu(buf, off, sess)
    assert results["more"].sum() > 0
    check(res, results, starts, buf, off, sess, "unsplit", allow_more=True)


def merged_split(seed):
    """A split coarser than the server's: runs of 1-3 consecutive server pieces
    merged, so a piece may hold several requests and the walk meets request
    boundaries inside pieces whose records an earlier request overwrote."""
    rng = np.random.default_rng(seed)

    def split(data):
        p, out = rhp.split_pieces(data), []
        while p:
            k = int(rng.integers(1, 4))
            out.append(sum(p[:k]))
            p = p[k:]
        return out
    return split


@pytest.mark.parametrize("emulate_dfa", [False, True])
def test_fixup_cpu_partly_merged_split(emulate_dfa):
    """Pieces that each hold up to three requests: requests past a
    piece's first are parsed again from their true boundary, never read from
    record slots the walk has already overwritten; sessions that run out of
    pieces report `more`."""
    data = make_sessions(80, 11)
    buf, off, sess, _ = rhp.pack_sessions(data, split=merged_split(11))
    res, results, starts = rhp.fixup_cpu(buf, off, sess, 16, emulate_dfa)
    check(res, results, starts, buf, off, sess, "merged", allow_more=True)


def test_fixup_cpu_every_chunking_of_one_stream():
    """One pipelined stream cut at every position into (delivered, rest): the
    delivered part as one session, as a server round sees a partial recv."""
    rng = np.random.default_rng(5)
    pool, _, _ = request_pool(rng)
    stream = b"".join(pool)
    data = [stream[:k] for k in range(0, len(stream) + 1, 7)]
    buf, off, sess, _ = rhp.pack_sessions(data)
    res, results, starts = rhp.fixup_cpu(buf, off, sess)
    check(res, results, starts, buf, off, sess, "prefixes")


@pytest.mark.gpu
@pytest.mark.parametrize("impl", [rhp.IMPL_DFA, rhp.IMPL_EXACT])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fixup_gpu_matches_reference_loop(seed, impl):
    data = make_sessions(400, seed)
    buf, off, sess, _ = rhp.pack_sessions(data)
    res, results, starts = rhp.fixup_gpu(buf, off, sess, 16, impl)
    total = check(res, results, starts, buf, off, sess, f"gpu impl{impl} seed {seed}")
    assert total > 400


@pytest.mark.gpu
def test_fixup_gpu_unsplit_sessions():
    data = make_sessions(200, 9)
    buf, off, sess, _ = rhp.pack_sessions(data, split=False)
    res, results, starts = rhp.fixup_gpu(buf, off, sess)
    assert results["more"].sum() > 0
    check(res, results, starts, buf, off, sess, "gpu unsplit", allow_more=True)


@pytest.mark.gpu
def test_fixup_gpu_partly_merged_split():
    data = make_sessions(300, 12)
    buf, off, sess, _ = rhp.pack_sessions(data, split=merged_split(12))
    res, results, starts = rhp.fixup_gpu(buf, off, sess)
    check(res, results, starts, buf, off, sess, "gpu merged", allow_more=True)


@pytest.mark.gpu
def test_fixup_gpu_prefixes():
    rng = np.random.default_rng(5)
    pool, _, _ = request_pool(rng)
    stream = b"".join(pool) * 3
    data = [stream[:k] for k in range(0, len(stream) + 1, 3)]
    buf, off, sess, _ = rhp.pack_sessions(data)
    res, results, starts = rhp.fixup_gpu(buf, off, sess)
    check(res, results, starts, buf, off, sess, "gpu prefixes")
