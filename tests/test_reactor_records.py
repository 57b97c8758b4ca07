"""What the server hands to SERVER_REQUEST, request by request, against the
oracle's sequential http_read_request loop over the same byte stream (the
reference's server_session_read loop, server.c:37-65, over http.c:177-234).

tests/reactor/echo_test.c serves one connection that sends a stream in chunks
(so rounds see partial requests and pipelined runs); its handler echoes the
parsed method, target, fields and body.  The oracle parses the stream from the
front, one request at a time, exactly as the reference's loop consumes it:
result 1 -> the request, advance by `consumed`; 0 -> wait (the tail gets no
answer); -1 -> the connection closes.  The streams mix pipelined GETs,
Content-Length and chunked bodies (de-framed in place), LF-only line ends,
HTTP/1.0, a request at the 16-field limit and bodies larger than a chunk.
Host parsers on CPU; the MI355X batch parser (asynchronous rounds) on the GPU.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

import libreactorng_amd as rhp
from oracle_util import run_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "libreactorng_amd", "bin", "echo_test")
TFB = (b"GET /plaintext HTTP/1.1\r\nHost: tfb-server:8080\r\nAccept: text/plain\r\n"
       b"Connection: keep-alive\r\nUser-Agent: wrk/4.2.0 (tfb-load)\r\n\r\n")


def stream_mixed(seed=7):
    rng = np.random.default_rng(seed)
    parts = [b"GET / HTTP/1.1\r\nHost: a\r\n\r\n",
             b"GET /path?q=1 HTTP/1.0\r\nA: 1\r\nB:  two words  \r\n\r\n",
             b"POST /body HTTP/1.1\r\nContent-Length: 5\r\n\r\nhello",
             b"POST /c HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n",
             b"GET /lf HTTP/1.1\nX: y\nZ:  w\n\n",
             b"GET /sixteen HTTP/1.1\r\n" + b"".join(b"H%d: v%d\r\n" % (i, i) for i in range(16)) + b"\r\n"]
    parts += [TFB] * 8
    big = bytes(rng.integers(97, 123, 3000, dtype=np.uint8))
    parts += [b"POST /big HTTP/1.1\r\nContent-Length: 3000\r\n\r\n" + big]
    parts += [b"PUT /chunked-hex HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n1a\r\n" + b"z" * 26 +
              b"\r\n0\r\n\r\n"]
    parts += [b"GET /t%d HTTP/1.1\r\nX-I: %d\r\n\r\n" % (i, i) for i in range(20)]
    parts += [b"GET /last HTTP/1.1\r\nHost:"]   # incomplete: no answer
    return b"".join(parts)


def stream_bad():
    return TFB * 3 + b"GET /x HTTP/1.1\r\nBad Header\r\n\r\n" + TFB


def oracle_sequential(stream: bytes, max_headers=16):
    """(method, target, fields, body) per request the reference's loop dispatches."""
    out, p = [], 0
    while p < len(stream):
        seg = stream[p:]
        buf = np.zeros(len(seg) + rhp.RHP_PAD, dtype=np.uint8)
        buf[: len(seg)] = np.frombuffer(seg, dtype=np.uint8)
        off = np.array([0, len(seg)], dtype=np.uint64)
        reqs, hdrs, http, rw = run_oracle(buf, off, max_headers, rhp.MODE_HTTP)
        res = int(http["result"][0])
        if res != 1:
            break
        r, b = reqs[0], bytes(rw[: len(seg)])
        fields = []
        for k in range(int(r["num_headers"])):
            h = hdrs[0][k]
            name = b"" if h["name_off"] < 0 else b[h["name_off"]: h["name_off"] + h["name_len"]]
            fields.append((name, b[h["value_off"]: h["value_off"] + h["value_len"]]))
        body = b""
        if http["body_kind"][0]:
            o = int(http["body_off"][0])
            body = b[o: o + int(http["body_len"][0])]
        out.append((b[r["method_off"]: r["method_off"] + r["method_len"]],
                    b[r["path_off"]: r["path_off"] + r["path_len"]], fields, body))
        p += int(http["consumed"][0])
    return out


def decode_echoes(raw: bytes):
    """Responses -> (method, target, fields, body) from echo_test's encoding."""
    out, p = [], 0
    while p < len(raw):
        end = raw.index(b"\r\n\r\n", p)
        head = raw[p:end].decode("latin-1")
        n = int([l for l in head.split("\r\n") if l.lower().startswith("content-length:")][0].split(":")[1])
        body = raw[end + 4: end + 4 + n]
        p = end + 4 + n
        q, items = 0, []
        while q < len(body):
            ln = struct.unpack_from("<I", body, q)[0]
            items.append(body[q + 4: q + 4 + ln])
            q += 4 + ln
        nf = struct.unpack("<I", items[2])[0]
        fields = [(items[3 + 2 * i], items[4 + 2 * i]) for i in range(nf)]
        out.append((items[0], items[1], fields, items[3 + 2 * nf]))
    return out


def run_echo(tmp_path, stream: bytes, chunk: int, parser: str, writer: str = "host"):
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    src.write_bytes(stream)
    p = subprocess.run([ECHO, str(src), str(chunk), str(dst)],
                       env=dict(os.environ, RHP_REACTOR_PARSER=parser, RHP_REACTOR_WRITER=writer),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout + p.stderr
    assert f"parser: {parser}" in p.stdout
    return decode_echoes(dst.read_bytes())


CASES = [("mixed", stream_mixed, 1 << 20), ("mixed", stream_mixed, 1000), ("mixed", stream_mixed, 61),
         ("mixed", stream_mixed, 7), ("bad", stream_bad, 1 << 20), ("bad", stream_bad, 50)]


def check_echoes(got, want, name, chunk):
    """A stream that ends in a malformed request: the reference closes the
    session in the same parse pass (server.c:47-51) and never reaches the
    stream_flush at the end of that pass (:64), so the replies to the requests
    parsed in that pass are never sent -- with the whole stream in one recv,
    none at all.  The echoes are the oracle's requests up to the last pass
    before the close: a prefix, all of it for well-formed streams."""
    if name == "bad":
        assert got == want[: len(got)]
        if chunk >= 1 << 20:
            assert got == []
    else:
        assert got == want


@pytest.mark.parametrize("parser,writer", [("host", "host"), ("host-async", "host"), ("host-async", "host-batch")])
@pytest.mark.parametrize("name,make,chunk", CASES)
def test_server_records_match_oracle_sequential_loop(tmp_path, name, make, chunk, parser, writer):
    s = make()
    want = oracle_sequential(s)
    assert len(want) >= 3
    check_echoes(run_echo(tmp_path, s, chunk, parser, writer), want, name, chunk)


@pytest.mark.gpu
@pytest.mark.parametrize("writer", ["host", "gpu"])
@pytest.mark.parametrize("name,make,chunk", CASES)
def test_server_records_gpu_match_oracle_sequential_loop(tmp_path, name, make, chunk, writer):
    """GPU parser (asynchronous rounds); replies written by the host as the
    reference does, or by rhp_write_responses once per round."""
    s = make()
    check_echoes(run_echo(tmp_path, s, chunk, "gpu", writer), oracle_sequential(s), name, chunk)


def stream_posts():
    """64 pipelined Content-Length POSTs and 16 chunked POSTs in one write (VERDICT r2
    'What's missing' 1): bodies end past their speculative pieces, one body holds
    empty lines and a whole fake request."""
    parts = []
    for i in range(64):
        body = b"b%03d" % i + (b"\r\n\r\nGET /fake HTTP/1.1\r\n\r\n" if i == 7 else b"")
        parts.append(b"POST /p%d HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % (i, len(body)) + body)
    for i in range(16):
        parts.append(b"POST /c%d HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nc%02d\r\n0\r\n\r\n" % (i, i))
    return b"".join(parts)


def rounds_of(tmp_path, stream, parser):
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    src.write_bytes(stream)
    p = subprocess.run([ECHO, str(src), str(1 << 20), str(dst)],
                       env=dict(os.environ, RHP_REACTOR_PARSER=parser, RHP_REACTOR_STATS="1"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout + p.stderr
    line = [l for l in p.stderr.splitlines() if l.startswith("server rounds:")][0]
    return int(line.split(":")[1].split(",")[0]), decode_echoes(dst.read_bytes())


@pytest.mark.parametrize("parser", ["host", "host-async"])
def test_pipelined_bodies_in_one_round(tmp_path, parser):
    s = stream_posts()
    rounds, got = rounds_of(tmp_path, s, parser)
    assert got == oracle_sequential(s)
    assert len(got) == 80
    assert rounds <= 2, rounds


@pytest.mark.gpu
def test_pipelined_bodies_in_one_round_gpu(tmp_path):
    s = stream_posts()
    rounds, got = rounds_of(tmp_path, s, "gpu")
    assert got == oracle_sequential(s)
    assert rounds <= 2, rounds


def stream_fake_chunked():
    """Content-Length bodies that hold whole chunked requests: the
    server's empty-line splitter makes pieces of them whose speculative parses
    are chunked requests, some complete within the bytes after them, that the
    fix-up absorbs into the body; real chunked requests around them are
    de-framed, so the round copies de-framed bytes back (reactor/batch.c walks
    only the record slots each session filled)."""
    fake = (b"POST /fake HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n4\r\nfake\r\n0\r\n\r\n")
    parts = []
    for i in range(12):
        body = b"x\r\n\r\n" + fake * (1 + i % 3) + b"tail%02d" % i
        parts.append(b"POST /cl%d HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % (i, len(body)) + body)
        parts.append(b"POST /ch%d HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n2\r\nc%d\r\n0\r\n\r\n" % (i, i % 10))
    parts.append(fake)   # a real one at the end
    return b"".join(parts)


@pytest.mark.parametrize("parser", ["host", "host-async"])
def test_fake_chunked_inside_bodies(tmp_path, parser):
    s = stream_fake_chunked()
    _, got = rounds_of(tmp_path, s, parser)
    want = oracle_sequential(s)
    assert len(want) == 25 and got == want


@pytest.mark.gpu
def test_fake_chunked_inside_bodies_gpu(tmp_path):
    s = stream_fake_chunked()
    _, got = rounds_of(tmp_path, s, "gpu")
    assert got == oracle_sequential(s)
