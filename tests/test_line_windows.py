"""phr mode's first windows start at the 128-byte line holding the request
(rhp_kernel.hip, window geometry): up to 127 bytes of the previous request lead
the window, zeroed and walked in S_PRE (rhp_dfa.h), and a request whose own first
byte is of the zeroed bytes' class (a CTL other than HT, LF, CR) goes to the exact
path.  These batches put request starts at every lead 0..127 with first bytes of
every kind and request lines/headers crossing the line boundary; the records must
equal the oracle's (picohttpparser.c:383-409) and the kernel's DFA / exact choice
(flags) the emulator's."""
import numpy as np
import pytest

import libreactorng_amd as rhp
from batches import pack
from oracle_util import assert_same, canon, run_oracle, to_rhp

FIRSTS = [b"GET / HTTP/1.1\r\nHost: a\r\nX-Long-Header-Name: " + b"v" * 90 + b"\r\n\r\n",
          b"POST /p HTTP/1.0\r\nA: b\r\n\r\n", b"\x00ET / HTTP/1.1\r\n\r\n", b"\x01GET / HTTP/1.1\r\n\r\n",
          b"\x7fGET / HTTP/1.1\r\n\r\n", b"\tGET / HTTP/1.1\r\n\r\n", b"\r\nGET / HTTP/1.1\r\n\r\n",
          b"\nGET / HTTP/1.1\r\n\r\n", b" GET / HTTP/1.1\r\n\r\n", b"\x80 / HTTP/1.1\r\n\r\n",
          b"G", b"", b"GET /" + b"a" * 200 + b" HTTP/1.1\r\nB: c\r\n\r\n"]


def lead_batch(reps=2, seed=3):
    """Request k starts at lead (k mod 128) of its line: each request is a base
    request plus filler after its end (bytes the parse never reaches) sized so the
    next one starts where wanted."""
    rng = np.random.default_rng(seed)
    reqs, pos = [], 0
    k = 0
    for _ in range(reps):
        for lead in range(128):
            for base in FIRSTS:
                body = bytearray(base)
                target_next = None
                # the next request's start: `lead` bytes past a line boundary after this request
                end = pos + len(body)
                target_next = ((end + 127) // 128) * 128 + (lead + 37 * k) % 128
                filler = target_next - end
                body += bytes(rng.integers(0x20, 0x7f, filler, dtype=np.uint8))
                reqs.append(bytes(body))
                pos += len(body)
                k += 1
    return pack(reqs)


def test_lead_batch_covers_every_lead():
    buf, off = lead_batch(reps=1)
    assert set((off[:-1] % 128).tolist()) == set(range(128))


@pytest.mark.parametrize("maxh", [0, 2, 16])
def test_line_windows_emulation_vs_oracle(maxh):
    buf, off = lead_batch()
    want = to_rhp(*run_oracle(buf, off, maxh, rhp.MODE_PHR)[:3], rhp.MODE_PHR)
    for layout in (rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_COMPACT):
        res, _ = rhp.emulate(buf, off, maxh, rhp.MODE_PHR, layout)
        assert_same(canon(res, rhp.MODE_PHR), want, buf, off, f"emulation, line windows, maxh {maxh}")
        first = buf[off[:-1].astype(np.int64)]
        ctl = ((first < 0x20) & (first != 9) & (first != 10) & (first != 13)) | (first == 0x7f)
        assert ((res.reqs["flags"][ctl] & rhp.F_EXACT) != 0).all(), "a CTL first byte takes the exact path"


@pytest.mark.gpu
@pytest.mark.parametrize("maxh", [0, 2, 16])
def test_gpu_line_windows_vs_oracle_and_emulator(maxh):
    buf, off = lead_batch()
    want = to_rhp(*run_oracle(buf, off, maxh, rhp.MODE_PHR)[:3], rhp.MODE_PHR)
    for layout in (rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_COMPACT):
        emu, _ = rhp.emulate(buf, off, maxh, rhp.MODE_PHR, layout)
        for impl in (rhp.IMPL_DFA, rhp.IMPL_DFA_LATE):
            res = rhp.parse_batch(buf, off, maxh, rhp.MODE_PHR, impl=impl, layout=layout)
            assert_same(canon(res, rhp.MODE_PHR), want, buf, off, f"GPU line windows impl{impl} maxh {maxh}")
            assert np.array_equal(res.reqs["flags"] & (rhp.F_EXACT | rhp.F_WIDE),
                                  emu.reqs["flags"] & (rhp.F_EXACT | rhp.F_WIDE)), (impl, layout)


def uneven_large_batch(n=1_300_000, seed=21):
    """Ranges of 4096-8192 requests (n / 256 CUs) whose first requests are longer
    than twice the range's mean: the longest-first hand-out with its order in
    the last TWO waves' staging (rhp_kernel.hip order_waves; 1M-request config 3
    ranges take one wave's).  Every 8th request carries 30 header lines, the
    rest are short; request starts fall at every lead."""
    rng = np.random.default_rng(seed)
    short = [b"GET /a HTTP/1.1\r\nH: v\r\n\r\n", b"POST /b HTTP/1.0\r\nA: 1\r\nB: 2\r\n\r\n", b"GET / HTTP/1.1\r\n\r\n"]
    long = b"GET /" + b"p" * 37 + b" HTTP/1.1\r\n" + b"".join(b"X-H%02d: %s\r\n" % (k, b"v" * (k % 7)) for k in range(30)) + b"\r\n"
    pick = rng.integers(0, len(short), n)
    reqs = [long if i % 8 == 0 else short[pick[i]] for i in range(n)]
    return pack(reqs)


@pytest.mark.gpu
def test_gpu_uneven_ranges_with_two_order_waves():
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    buf, off = uneven_large_batch(n=cus * 5000)
    assert 4096 < (len(off) - 1) // cus <= 8192
    want = to_rhp(*run_oracle(buf, off, 32, rhp.MODE_PHR)[:3], rhp.MODE_PHR)
    res = rhp.parse_batch(buf, off, 32, rhp.MODE_PHR)
    assert_same(canon(res, rhp.MODE_PHR), want, buf, off, "GPU uneven ranges, two order waves")
