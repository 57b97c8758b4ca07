"""Hand-built request batches shared by the CPU and GPU tests and by
tests/golden/make_golden.py (builder sets): the batch contract's edge cases,
dense header lines, and inputs longer than 64 KiB."""
from __future__ import annotations

import numpy as np

import libreactorng_amd as rhp


def pack(reqs, pad=rhp.RHP_PAD, align_shift=0):
    parts = [bytes(r) for r in reqs]
    off = np.zeros(len(parts) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(p) for p in parts])
    off += align_shift
    buf = np.zeros(int(off[-1]) + pad, dtype=np.uint8)
    buf[align_shift:int(off[-1])] = np.frombuffer(b"".join(parts), dtype=np.uint8)
    return buf, off


EDGE = [
    b"", b"G", b"GET", b"GET ", b"GET  ", b" ", b"GET /", b"GET / ", b"\r", b"\n", b"\r\n", b"\r\nGET ",
    b"GET / HTTP/1.1\r\n\r\n", b"GET / HTTP/1.1\n\n", b"\r\nGET / HTTP/1.1\r\n\r\n", b"\nGET / HTTP/1.0\n\n",
    b"GET / HTTP/1.10\r\n\r\n", b"GET / HTTP/1.1\r\nA: b\r\n \tfolded  \r\n\r\n", b"GET / HTTP/1.1\r\nA :b\r\n\r\n",
    b"GET / HTTP/1.1\r\n:b\r\n\r\n", b"GET / HTTP/1.1\r\nA:\r\n\r\n", b"GET / HTTP/1.1\r\nA: \t \r\n\r\n",
    b"GET / HTTP/1.1\r\nA: x \t\r\n\r\n", b"GET / HTTP/1.1\r\nA: \x80\xff \r\n\r\n", b"GET / HTTP/1.1\r\nA: a\rb\r\n\r\n",
    b"GET / HTTP/1.1\r\nA: a\x7fb\r\n\r\n", b"GET \x80\xfe HTTP/1.1\r\n\r\n", b"\x80 / HTTP/1.1\r\n\r\n",
    b"GET / HTTP/1.1\r\n\r\nGET / HTTP/1.1\r\n\r\n", b"POST / HTTP/1.1\r\nContent-Length: 3\r\n\r\nabc",
    b"GET / HTTP/1.1\r", b"GET / HTTP/1.1\r\nA: b\r", b"GET / HTTP/1.1\r\nA: b\r\n\r",
    b"  / HTTP/1.1\r\n\r\n", b"GET  /  HTTP/1.1\r\n\r\n", b"GET / H\r\n\r\n",
]


def version_batch():
    """Request lines whose version is not HTTP/1.<digit>, cut at every length: the
    kernel's DFA answers -1 for them only when the version's 9 bytes are in the
    buffer (picohttpparser.c:248-258, rhp_dfa.h S_V1..S_V7), else the exact path
    decides (-2 for a short buffer)."""
    bases = [b"GET / HTTP/2.0\r\n\r\n", b"GET / HTTX/1.1\r\nA: b\r\n\r\n", b"GET / XTTP/1.1\r\n\r\n",
             b"GET / HTTP/1.x\r\n\r\n", b"GET / HTTP/1.5\r\n\r\n", b"GET / HTTP/11.1\r\n\r\n",
             b"GET / http/1.1\r\n\r\n", b"GET /p \r\n\r\n", b"GET /p HTTP/1.1X\r\n\r\n", b"GET /p HTTP/1.\x01\r\n\r\n",
             b"POST /u HTTP/2.0\r\nContent-Length: 3\r\n\r\nabc", b"GET /p HTTP/1.1\rX\r\n\r\n"]
    return [b[:k] for b in bases for k in range(len(b) + 1)]


def dense_header_batch(n=3000, seed=5):
    """Adversarial: many 3-byte header lines ("a:\n") so up to 6 header records
    start inside one 16-byte check interval (capture-ring wrap, request-line
    clobber rule, flush ordering; rhp_dfa.h)."""
    rng = np.random.default_rng(seed)
    reqs = []
    for _ in range(n):
        rl = (b"GET /" + b"p" * int(rng.integers(0, 40)) + b" HTTP/1." + bytes([48 + int(rng.integers(0, 10))]) +
              (b"\r\n" if rng.random() < .5 else b"\n"))
        hs = b"".join((b"a:\n" if rng.random() < .6 else b"bb: v \r\n" if rng.random() < .5 else b"c:\r\n")
                      for _ in range(int(rng.integers(0, 40))))
        reqs.append(rl + hs + (b"\r\n" if rng.random() < .9 else b""))
    return reqs


def long_batch():
    """Inputs longer than 64 KiB: bodies and pipelines past
    the u16 record range are parsed exactly; only a header section longer than
    65535 B is RHP_RET_TOOLONG.  Reference: http.c:177-234 (no size limit),
    buffer.c:56-64 (buffers grow without bound)."""
    def post(n):
        return b"POST /upload HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % n
    get = b"GET /plaintext HTTP/1.1\r\nHost: tfb\r\n\r\n"
    chunks = b"".join(b"%x\r\n%s\r\n" % (4000, b"c" * 4000) for _ in range(20)) + b"0\r\n\r\n"
    return [
        post(200000) + b"x" * 200000,                       # 200 KB Content-Length POST
        post(1 << 20) + b"y" * (1 << 20),                   # 1 MiB POST
        post(200000) + b"x" * 150000,                       # body still arriving -> http 0
        get * (72000 // len(get)),                          # ~70 KiB of pipelined GETs
        get + b"\x00" * 70000,                              # 70 KB after a complete GET
        b"GET /" + b"a" * 70000 + b" HTTP/1.1\r\n\r\n",      # header section > 64 KiB: TOOLONG
        b"GET / HTTP/1.1\r\nX: " + b"v" * 70000 + b"\r\n\r\n",  # ... in a value: TOOLONG
        b"GET / HTTP/1.1\r\nX: " + b"v" * 70000,              # incomplete past 64 KiB -> -2
        b"GET / HTTP/1.1\r\nX: " + b"v" * 70000 + b"\x01\r\n\r\n",  # CTL past 64 KiB -> -1
        b"GET / HTTP/1.1\r\n" + b"".join(b"H%d: %s\r\n" % (i, b"z" * 5000) for i in range(20)) + b"\r\n",
        b"POST /c HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n" + chunks,   # 80 KB chunked body
        b"POST /c HTTP/1.1\r\nContent-Length: 70000\r\n\r\n" + b"b" * 69999,   # one byte short -> 0
        b"PUT /q HTTP/1.0\r\nContent-Length: 99999999999999999999999\r\n\r\n" + b"q" * 66000,
    ]


BUILDERS = {"long_batch": long_batch, "edge": lambda: EDGE * 3, "dense": lambda: dense_header_batch(2000, 21)}


def chunked_paths_batch(n=6000, seed=11):
    """Chunked POSTs that take every path of the GPU replay's de-framing
    (rhp_kernel.hip ChunkWalk / staged_moves / DevMove): 1-8 chunks in a slot
    (staged), chunks of 1-15 bytes (a block drawing on three or more chunks),
    9-24 chunks (moved by the lane, second walk), 1-8 chunks beyond a 2 KiB slot
    (moved by the lane from the kept spans), size lines longer than the 17-20
    byte window (extensions, OWS, leading zeros), bodies that end at the request's
    end (the last line reaches into the next request: byte stores), malformed and
    partial framing, and plain requests between them."""
    import random
    rng = random.Random(seed)
    data = np.random.default_rng(seed).integers(33, 127, size=1 << 20, dtype=np.uint8).tobytes()
    out = []

    def payload(sz):
        at = rng.randrange(0, len(data) - sz)
        return data[at:at + sz]

    def size_line(sz):
        h = f"{sz:x}" if rng.random() < 0.7 else f"{sz:X}"
        r = rng.random()
        if r < 0.08:
            h = "0" * rng.randrange(1, 20) + h   # long line: leading zeros
        elif r < 0.14:
            h = " " * rng.randrange(1, 4) + h + "\t" * rng.randrange(0, 3)
        elif r < 0.22:
            h = h + ";name=" + "v" * rng.randrange(0, 40)   # extension, sometimes past the window
        return h.encode() + b"\r\n"

    for i in range(n):
        kind = rng.randrange(10)
        if kind == 0:
            out.append(b"GET /g HTTP/1.1\r\nHost: a\r\n\r\n")
            continue
        if kind == 1:
            sizes = [rng.randrange(1, 16) for _ in range(rng.randrange(3, 9))]          # tiny chunks
        elif kind == 2:
            sizes = [rng.randrange(1, 200) for _ in range(rng.randrange(9, 25))]        # many chunks
        elif kind == 3:
            sizes = [rng.randrange(300, 900) for _ in range(rng.randrange(3, 8))]       # beyond a slot
        else:
            sizes = [rng.randrange(1, 400) for _ in range(rng.randrange(1, 9))]         # staged
        body = b"".join(size_line(s) + payload(s) + b"\r\n" for s in sizes)
        tail = b"0\r\n\r\n"
        r = rng.random()
        if r < 0.04:
            body = body.replace(b"\r\n", b"\n", 1)            # bare LF after a size line
        elif r < 0.08:
            body = b"zz\r\n" + body                            # not hex
        elif r < 0.12:
            tail = b""                                         # partial: no last chunk
        elif r < 0.14:
            tail = b"0;last\n\r\n"
        head = b"POST /u HTTP/1.1\r\nHost: h\r\nTransfer-Encoding: " + rng.choice([b"chunked", b"Chunked", b"CHUNKED"]) + b"\r\n\r\n"
        out.append(head + body + tail)
    return out
