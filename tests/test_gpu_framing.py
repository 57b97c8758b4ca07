"""GPU parity of http_read_request's framing (/root/reference/src/reactor/http.c:196-218)
as the late-issue DFA kernel evaluates it inside its loop: the first
Transfer-Encoding / Content-Length candidate is read from the staging buffer
while its window is there, a Content-Length value that crosses a window
boundary is carried as a number into the next window, and everything else
(several candidates, chunked, long values, names that start in an earlier
window) is left to the replay.  Each case slides the framing header across the
128-byte window boundaries (a padding header of every length in front of it)
and starts requests at every alignment; expected results come from the oracle
(oracle/rhp_oracle.c, pinned to the compiled reference by tests/golden)."""
import numpy as np
import pytest

import libreactorng_amd as rhp
from batches import pack
from oracle_util import assert_same, canon, run_oracle, to_rhp

pytestmark = pytest.mark.gpu

# (framing header lines, body) variants: the single Content-Length case the
# kernel frames itself, and the cases it must decline or get exactly right
VARIANTS = [
    (b"Content-Length: 5\r\n", b"abcde"),
    (b"content-length: 12\r\n", b"x" * 12),
    (b"CONTENT-LENGTH: 0\r\n", b""),
    (b"Content-Length: 007\r\n", b"1234567"),
    (b"Content-Length: +3\r\n", b"abc"),
    (b"Content-Length: -1\r\n", b"zz"),                      # strtoull wraps: result 0
    (b"Content-Length: 4x9\r\n", b"abcd"),                   # digits stop at 'x'
    (b"Content-Length: 99999999999\r\n", b"q"),             # longer than the input: result 0
    (b"Content-Length: 1234567890123456789\r\n", b"q"),     # 19 digits
    (b"Content-Length: 12345678901234567890123\r\n", b"q"), # saturates (replay)
    (b"Content-Length: \r\n", b"abc"),                       # empty value: no body
    (b"Content-Lengtx: 5\r\n", b"abcde"),                    # a 14-byte name that is not CL
    (b"Accept-Charset: 5\r\n", b"abcde"),
    (b"If-Modified-Since: 5\r\n", b"abcde"),                 # a 17-byte name that is not TE
    (b"Transfer-Encoding: chunked\r\n", b"3\r\nabc\r\n0\r\n\r\n"),
    (b"Transfer-Encoding: gzip\r\n", b"abc"),
    (b"Transfer-Encoding: \r\nContent-Length: 2\r\n", b"ab"),
    (b"Content-Length: 2\r\nTransfer-Encoding: chunked\r\n", b"ab"),
    (b"Content-Length: 2\r\nContent-Length: 3\r\n", b"abc"),
    (b"Accept-Charset: 1\r\nContent-Length: 3\r\n", b"abc"),
    # two candidates, settled in the replay's first pass
    (b"Transfer-Encoding: chunked\r\nContent-Length: 3\r\n", b"abc"),
    (b"Content-Length: \r\nTransfer-Encoding: chunked\r\n", b"3\r\nabc\r\n0\r\n\r\n"),
    (b"Content-Length: \r\nContent-Length: 3\r\n", b"abc"),      # the first CL counts, empty
    (b"Transfer-Encoding: chunked\r\nTransfer-Encoding: gzip\r\n", b"3\r\nabc\r\n0\r\n\r\n"),
    (b"Transfer-Encoding: gzip\r\nTransfer-Encoding: chunked\r\n", b"abc"),
    (b"If-Modified-Since: 1\r\nContent-Length: 3\r\n", b"abc"),
    (b"Transfer-Encoding: CHUNKED\r\nIf-Modified-Since: x\r\n", b"3\r\nabc\r\n0\r\n\r\n"),
    (b"Content-Lengtx: 9\r\nContent-Length: 12345678901234567890123\r\n", b"q"),
    (b"Accept-Charset: 1\r\nIf-Modified-Since: 2\r\n", b"abc"),   # neither is framing
    # three candidates: the general path
    (b"Content-Length: 3\r\nAccept-Charset: x\r\nTransfer-Encoding: chunked\r\n", b"abc"),
    (b"Accept-Charset: x\r\nAccept-Charset: y\r\nContent-Length: 3\r\n", b"abc"),
]


def requests(seed):
    rng = np.random.default_rng(seed)
    reqs = []
    for hdr, body in VARIANTS:
        for pad in range(0, 150, 1):
            method = b"POST" if rng.random() < .9 else b"GET"
            pre = b"%s /u HTTP/1.1\r\nX-Pad: %s\r\n" % (method, b"p" * pad)
            tail = b"" if rng.random() < .9 else b"Host: h\r\n"
            r = pre + hdr + tail + b"\r\n" + body
            if rng.random() < .1:
                r = r[:int(rng.integers(len(pre), len(r) + 1))]   # truncated: partial or short body
            reqs.append(r)
    order = rng.permutation(len(reqs))
    return [reqs[i] for i in order]


@pytest.mark.parametrize("layout", [rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_HEADER_MAJOR])
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_gpu_framing_across_windows(layout, shift):
    reqs = requests(100 + shift)
    buf, off = pack(reqs, align_shift=shift)
    for maxh in (16, 2):
        res = rhp.parse_batch(buf, off, maxh, rhp.MODE_HTTP, layout=layout)
        want = to_rhp(*run_oracle(buf, off, maxh, rhp.MODE_HTTP)[:3], rhp.MODE_HTTP)
        assert_same(canon(res, rhp.MODE_HTTP), want, buf, off, f"framing shift{shift} maxh{maxh}")


def test_gpu_framing_many_per_workgroup():
    """Enough requests that every workgroup's deferred list (480 entries) both
    fits and overflows in one batch: the replay takes the list or the range."""
    reqs = requests(7) * 40
    rng = np.random.default_rng(8)
    # a stretch of chunked requests, all deferred, somewhere in the batch
    chunked = [b"POST /c HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n2\r\nab\r\n0\r\n\r\n"] * 6000
    at = int(rng.integers(0, len(reqs)))
    reqs = reqs[:at] + chunked + reqs[at:]
    buf, off = pack(reqs)
    res = rhp.parse_batch(buf, off, 16, rhp.MODE_HTTP, layout=rhp.LAYOUT_HEADER_MAJOR)
    want = to_rhp(*run_oracle(buf, off, 16, rhp.MODE_HTTP)[:3], rhp.MODE_HTTP)
    assert_same(canon(res, rhp.MODE_HTTP), want, buf, off, "framing many")
