"""libreactorng_amd -- MI355X-native batched HTTP/1.1 request parser (rhp).

Python plumbing over the C-ABI in include/rhp.h (librhp.so, HIP/gfx950) and the
host helpers in include/rhp_gen.h (librhp_host.so).  The product path is the HIP
kernel: `parse_batch` raises if librhp.so is missing or no GPU is visible; it
never falls back to a CPU parser.

Reference interface mirrored (record fields are offsets from each request start):
  phr_parse_request   /root/reference/src/picohttpparser/picohttpparser.h:51-52
  http_read_request   /root/reference/src/reactor/http.h:36
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIBRHP = os.environ.get("RHP_LIB", os.path.join(_HERE, "librhp.so"))  # RHP_LIB: A/B experiments only
LIBHOST = os.path.join(_HERE, "librhp_host.so")

RHP_PAD = 256
RHP_MAX_LEN = 65535
RHP_MAX_HEADERS = 64
RHP_RET_TOOLONG = -3
RHP_WORK_WORDS = 64
MODE_PHR, MODE_HTTP = 0, 1
LAYOUT_REQUEST_MAJOR, LAYOUT_HEADER_MAJOR, LAYOUT_COMPACT, LAYOUT_DENSE, LAYOUT_DENSE_RM = 0, 1, 2, 3, 4
DENSE_LAYOUTS = (LAYOUT_DENSE, LAYOUT_DENSE_RM)            # rhp.h: 8-byte request records, u16 lengths
LENGTH_LAYOUTS = (LAYOUT_COMPACT,) + DENSE_LAYOUTS          # records expanded by the running sum
IMPL_DFA, IMPL_EXACT, IMPL_DFA_LATE = 0, 1, 2
RHP_NAME_NULL = 0xFFFF
F_EXACT = 0x1
F_WIDE = 0x2   # compact layout: the request's header records are in the wide area (rhp.h)
HTTP_WIDE = 0x1   # compact http records (rhp_http_compact_t.flags): the record is in the wide area (rhp.h)
DENSE_WIDE, DENSE_BAD = 0x1, 0x2   # dense request records (rhp_req_dense_t.flags, rhp.h)

GEN_TFB128, GEN_GET256, GEN_ZIPF, GEN_POST1K, GEN_CHUNKED, GEN_FUZZ, GEN_FUZZ_HTTP = 1, 2, 3, 5, 6, 100, 101

# numpy views of the C records (rhp.h)
REQ_DTYPE = np.dtype([("ret", "<i4"), ("method_len", "<u2"), ("path_off", "<u2"), ("path_len", "<u2"),
                      ("method_off", "u1"), ("minor_version", "i1"), ("num_headers", "<u2"),
                      ("flags", "<u2")])
HDR_DTYPE = np.dtype([("name_off", "<u2"), ("name_len", "<u2"), ("value_off", "<u2"), ("value_len", "<u2")])
HTTP_DTYPE = np.dtype([("result", "<i4"), ("body_kind", "<u4"), ("consumed", "<u8"), ("body_len", "<u8")])
assert REQ_DTYPE.itemsize == 16 and HDR_DTYPE.itemsize == 8 and HTTP_DTYPE.itemsize == 24


class Batch(ctypes.Structure):
    """struct rhp_batch (include/rhp.h)."""
    _fields_ = [("bytes", ctypes.c_void_p), ("bytes_rw", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("bytes_size", ctypes.c_uint64), ("n", ctypes.c_uint32), ("max_headers", ctypes.c_uint32),
                ("mode", ctypes.c_uint32), ("layout", ctypes.c_uint32), ("reqs", ctypes.c_void_p),
                ("hdrs", ctypes.c_void_p), ("http", ctypes.c_void_p), ("work", ctypes.c_void_p),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("last_len", ctypes.c_void_p)]


BATCH_SPECULATIVE = 1        # rhp_batch_t.flags (rhp.h RHP_BATCH_SPECULATIVE)
BODY_CHUNKED_PENDING = 2
SESSION_DTYPE = np.dtype([("piece_lo", "<u4"), ("piece_hi", "<u4")])
SESSION_RESULT_DTYPE = np.dtype([("n_slots", "<u4"), ("more", "<u4"), ("consumed", "<u8")])


# exported C-ABI symbols of librhp.so, as declared in include/rhp.h
RHP_SYMBOLS = ("rhp_parse_batch", "rhp_set_impl", "rhp_kernel_name", "rhp_version", "rhp_write_responses",
               "rhp_fixup_sessions", "rhp_pack_dense")
HOST_SYMBOLS = ("rhp_gen_size", "rhp_gen_fill", "rhp_gen_header_bytes", "rhp_splitmix64",
                "rhp_emu_parse_batch", "rhp_cpu_parse_batch", "rhp_phr_parse_request", "rhp_http_read_cpu",
                "rhp_cpu_fixup_sessions", "rhp_expand_records", "rhp_expand_http", "rhp_expand_reqs", "rhp_cpu_pack_dense",
                "rhp_test_chunk_window",
                "rhp_test_chunk_exact")

_rhp = None
_host = None


class RespBatch(ctypes.Structure):
    """rhp_resp_batch_t (include/rhp.h): http_write_response over a batch"""
    _fields_ = [("arena", ctypes.c_void_p), ("resps", ctypes.c_void_p), ("fields", ctypes.c_void_p),
                ("n", ctypes.c_uint32), ("date_len", ctypes.c_uint32), ("date", ctypes.c_char_p),
                ("out_off", ctypes.c_void_p), ("out", ctypes.c_void_p), ("out_size", ctypes.c_uint64),
                ("work", ctypes.c_void_p)]


RHP_DATE_LEN = 29


def _torch_hip_runtime() -> str | None:
    """Path of the HIP runtime torch ships (torch/lib/libamdhip64.so), found
    without importing torch."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    path = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    return path if os.path.exists(path) else None


def hip_runtimes() -> list[str]:
    """The libamdhip64 files mapped into this process (Linux /proc/self/maps)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln and "/" in ln})
    except OSError:
        return []


def check_one_hip_runtime() -> None:
    """Two HIP runtimes in one process (torch's and /opt/rocm's) each own their
    device memory: a kernel of one launched on buffers of the other fails with
    error 100.  Raise with the cause instead."""
    rt = [os.path.realpath(p) for p in hip_runtimes()]
    if len(set(rt)) > 1:
        raise RuntimeError("two HIP runtimes are loaded (" + ", ".join(sorted(set(rt))) + "): librhp.so was "
                           "loaded before torch without libreactorng_amd.lib(); load it through lib(), or "
                           "import torch first")


def lib() -> ctypes.CDLL:
    """librhp.so (HIP).  Raises if it is missing: there is no fallback.

    Load order.  librhp.so's DT_NEEDED is libamdhip64.so.7 (the
    soname of both /opt/rocm's runtime and the one torch ships); torch's
    libc10_hip.so asks for the unversioned libamdhip64.so through its $ORIGIN
    rpath.  ld.so reuses a loaded library only when a request matches its soname
    or the name it was loaded by, so torch-first gives one runtime (librhp's
    request matches the soname of torch's copy), while librhp-first loads
    /opt/rocm's copy and torch's later request for `libamdhip64.so` matches
    neither name: torch then loads its own copy, and tensors it allocates are
    foreign to librhp's runtime.  So torch's runtime, when torch is installed, is
    preloaded by path (RTLD_GLOBAL) before librhp.so, without importing torch;
    a process without torch uses /opt/rocm's."""
    global _rhp
    if _rhp is None:
        if not os.path.exists(LIBRHP):
            raise RuntimeError(f"{LIBRHP} missing: run __graft_entry__.build() (hipcc gfx950)")
        rt = _torch_hip_runtime()
        if rt is not None:
            ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)
        _rhp = ctypes.CDLL(LIBRHP)
        check_one_hip_runtime()
        _rhp.rhp_parse_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p]
        _rhp.rhp_parse_batch.restype = ctypes.c_int
        _rhp.rhp_set_impl.argtypes = [ctypes.c_int]
        _rhp.rhp_set_impl.restype = ctypes.c_int
        _rhp.rhp_kernel_name.restype = ctypes.c_char_p
        _rhp.rhp_version.restype = ctypes.c_char_p
        _rhp.rhp_write_responses.argtypes = [ctypes.POINTER(RespBatch), ctypes.c_void_p]
        _rhp.rhp_write_responses.restype = ctypes.c_int
        vp = ctypes.c_void_p
        _rhp.rhp_pack_dense.argtypes = [ctypes.POINTER(Batch), vp, vp, vp, vp]
        _rhp.rhp_pack_dense.restype = ctypes.c_int
    return _rhp


def host() -> ctypes.CDLL:
    """librhp_host.so: generator, CPU exact parser, DFA emulator."""
    global _host
    if _host is None:
        if not os.path.exists(LIBHOST):
            raise RuntimeError(f"{LIBHOST} missing: run __graft_entry__.build()")
        _host = ctypes.CDLL(LIBHOST)
        u64 = ctypes.c_uint64
        _host.rhp_gen_size.argtypes = [ctypes.c_int, u64, u64, u64]
        _host.rhp_gen_size.restype = u64
        _host.rhp_gen_fill.argtypes = [ctypes.c_int, u64, u64, u64, ctypes.c_void_p, ctypes.c_void_p]
        _host.rhp_gen_fill.restype = ctypes.c_int
        _host.rhp_gen_header_bytes.argtypes = [ctypes.c_int, u64, u64, u64]
        _host.rhp_gen_header_bytes.restype = u64
        _host.rhp_emu_parse_batch.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p]
        _host.rhp_emu_parse_batch.restype = ctypes.c_int
        _host.rhp_cpu_parse_batch.argtypes = [ctypes.POINTER(Batch)]
        _host.rhp_cpu_parse_batch.restype = ctypes.c_int
        sz, vp = ctypes.c_size_t, ctypes.c_void_p
        P = ctypes.POINTER
        _host.rhp_phr_parse_request.argtypes = [vp, sz, P(vp), P(sz), P(vp), P(sz), P(ctypes.c_int),
                                                P(PhrHeader), P(sz), sz]
        _host.rhp_phr_parse_request.restype = ctypes.c_int
        _host.rhp_http_read_cpu.argtypes = [vp, sz, P(HttpReq), P(PhrHeader), P(sz)]
        _host.rhp_http_read_cpu.restype = ctypes.c_int
        _host.rhp_cpu_fixup_sessions.argtypes = [ctypes.POINTER(Batch), vp, ctypes.c_uint32, vp, vp]
        _host.rhp_cpu_fixup_sessions.restype = ctypes.c_int
        _host.rhp_expand_records.argtypes = [ctypes.POINTER(Batch), vp, vp, vp]
        _host.rhp_expand_records.restype = ctypes.c_int
        _host.rhp_expand_http.argtypes = [ctypes.POINTER(Batch), vp, vp, vp]
        _host.rhp_expand_reqs.argtypes = [ctypes.POINTER(Batch), vp, vp]
        _host.rhp_cpu_pack_dense.argtypes = [ctypes.POINTER(Batch), vp, vp, vp]
        _host.rhp_cpu_pack_dense.restype = ctypes.c_int
        _host.rhp_expand_reqs.restype = ctypes.c_int
        _host.rhp_expand_http.restype = ctypes.c_int
    return _host


class PhrHeader(ctypes.Structure):
    """struct phr_header (picohttpparser.h:42-47) = rhp_phr_header_t (include/rhp_host.h)."""
    _fields_ = [("name", ctypes.c_void_p), ("name_len", ctypes.c_size_t), ("value", ctypes.c_void_p),
                ("value_len", ctypes.c_size_t)]


class HttpReq(ctypes.Structure):
    """rhp_http_req_t (include/rhp_host.h)."""
    _fields_ = [("method", ctypes.c_void_p), ("method_len", ctypes.c_size_t), ("target", ctypes.c_void_p),
                ("target_len", ctypes.c_size_t), ("minor_version", ctypes.c_int), ("body", ctypes.c_void_p),
                ("body_len", ctypes.c_size_t), ("consumed", ctypes.c_uint64)]


def phr_parse_request_cpu(buf: np.ndarray, start: int, length: int, max_headers: int, last_len: int = 0):
    """rhp_phr_parse_request (the host drop-in for phr_parse_request) on bytes
    buf[start:start+length] (buf may be read past the end, as the reference does).
    Returns (ret, minor, method(off,len), path(off,len), [(name_off|-1, name_len,
    value_off, value_len)]) with offsets from `start`."""
    h = host()
    hdrs = (PhrHeader * max(max_headers, 1))()
    m, pth = ctypes.c_void_p(), ctypes.c_void_p()
    ml, pl, nh = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t(max_headers)
    minor = ctypes.c_int()
    base = buf.ctypes.data + start
    ret = h.rhp_phr_parse_request(base, length, ctypes.byref(m), ctypes.byref(ml), ctypes.byref(pth),
                                  ctypes.byref(pl), ctypes.byref(minor), hdrs, ctypes.byref(nh), last_len)
    if ret <= 0:
        return ret, -1, (0, 0), (0, 0), []
    rel = lambda p: (p or 0) - base
    hs = [(rel(x.name) if x.name else -1, x.name_len, rel(x.value), x.value_len) for x in hdrs[: nh.value]]
    return ret, minor.value, (rel(m.value), ml.value), (rel(pth.value), pl.value), hs


def http_read_cpu(buf: np.ndarray, start: int, length: int, max_headers: int = 16):
    """rhp_http_read_cpu (http_read_request with pointer outputs) on buf[start:start+length]
    (written in place for chunked bodies).  Returns (result, consumed, body(off,len) | None)."""
    h = host()
    hdrs = (PhrHeader * max(max_headers, 1))()
    r = HttpReq()
    nh = ctypes.c_size_t(max_headers)
    base = buf.ctypes.data + start
    res = h.rhp_http_read_cpu(base, length, ctypes.byref(r), hdrs, ctypes.byref(nh))
    if res != 1:
        return res, 0, None
    body = (r.body - base, r.body_len) if r.body else None
    return res, int(r.consumed), body


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def generate(config: int, n: int, seed: int, lo: int = 0):
    """Requests [lo, lo+n) of a generator config -> (bytes uint8[size+RHP_PAD], offsets uint64[n+1])."""
    h = host()
    size = h.rhp_gen_size(config, lo, lo + n, seed)
    if size == 0 and n > 0 and config not in (GEN_FUZZ, GEN_FUZZ_HTTP):
        raise ValueError(f"bad generator config {config}")
    buf = np.zeros(size + RHP_PAD, dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint64)
    if h.rhp_gen_fill(config, lo, lo + n, seed, _ptr(buf), _ptr(off)) != 0:
        raise ValueError(f"generator failed for config {config}")
    return buf, off


def header_bytes(config: int, n: int, seed: int, lo: int = 0) -> int:
    """Algorithmic bytes of requests [lo, lo+n)."""
    return int(host().rhp_gen_header_bytes(config, lo, lo + n, seed))


@dataclass
class Result:
    reqs: np.ndarray           # REQ_DTYPE [n]
    hdrs: np.ndarray           # HDR_DTYPE [n, max_headers] (a view of the header-major batch array; the
    #                            compact layout's records expanded by rhp_expand_records)
    http: np.ndarray | None    # HTTP_DTYPE [n] (http mode)
    bytes_out: np.ndarray | None = None  # request bytes after http mode (chunked bodies rewritten)
    raw_hdrs: np.ndarray | None = None   # the hdrs buffer as the parser left it (its layout's bytes)
    raw_http: np.ndarray | None = None   # the http buffer as the parser left it (compact: rhp_http_compact_t)
    raw_reqs: np.ndarray | None = None   # the reqs buffer as the parser left it (dense: rhp_req_dense_t + wide)


def canonical(res: Result, mode: int):
    """Result -> canonical (reqs, hdrs[n, max_headers], http) records: the fields
    the reference leaves unspecified for a request that did not parse (its
    method/path/header outputs, phr_parse_request's minor_version, the records
    past num_headers, flags) zeroed, so two parsers compare with one array
    equality and hash to one digest (tests/golden/full_digests.json)."""
    reqs = res.reqs.copy()
    n = len(reqs)
    maxh = res.hdrs.shape[1] if res.hdrs.ndim == 2 else 0
    ok = reqs["ret"] > 0
    if mode == MODE_HTTP:
        ok &= res.http["result"] == 1
    for f in ("method_off", "method_len", "path_off", "path_len", "num_headers"):
        reqs[f][~ok] = 0
    reqs["minor_version"][~ok] = -1
    reqs["flags"] = 0
    h = res.hdrs.copy() if maxh else np.zeros((n, 0), dtype=HDR_DTYPE)   # C order (header-major views too)
    if maxh:
        valid = ok[:, None] & (np.arange(maxh)[None, :] < reqs["num_headers"][:, None])
        for f in h.dtype.names:
            h[f] = np.where(valid, h[f], 0)
    x = None
    if mode == MODE_HTTP:
        x = res.http.copy()
        one = x["result"] == 1
        for f in ("body_kind", "consumed", "body_len"):
            x[f][~one] = 0
    return reqs, h, x


def record_digest(reqs, hdrs, http=None) -> str:
    """sha256 of a canonical record stream: reqs, then hdrs (request-major), then http."""
    import hashlib
    d = hashlib.sha256()
    d.update(np.ascontiguousarray(reqs).tobytes())
    d.update(np.ascontiguousarray(hdrs).tobytes())
    if http is not None:
        d.update(np.ascontiguousarray(http).tobytes())
    return d.hexdigest()


def library_sha256(path: str | None = None) -> str:
    """sha256 of librhp.so as it lies on disk (the file lib() loads): logs and
    profiles carry it so a result can be tied to the binary it came from."""
    import hashlib
    p = path or LIBRHP
    if not os.path.exists(p):
        return "missing"
    return hashlib.sha256(open(p, "rb").read()).hexdigest()


def hdrs_bytes(n: int, max_headers: int, layout: int) -> int:
    """bytes the batch's hdrs buffer needs (rhp.h; RHP_COMPACT_HDRS_BYTES / RHP_DENSE_HDRS_BYTES)"""
    if layout == LAYOUT_COMPACT:
        return ((n * max_headers * 4 + 15) & ~15) + n * max_headers * HDR_DTYPE.itemsize
    if layout in DENSE_LAYOUTS:   # u16 lengths, the u32 overflow area, the wide records
        return ((n * max_headers * 2 + 15) & ~15) + ((n * max_headers * 4 + 15) & ~15) + n * max_headers * HDR_DTYPE.itemsize
    return n * max_headers * HDR_DTYPE.itemsize


def reqs_bytes(n: int, layout: int) -> int:
    """bytes the batch's reqs buffer needs (rhp.h; RHP_DENSE_REQS_BYTES for the dense layout)"""
    if layout in DENSE_LAYOUTS:
        return ((n * 8 + 15) & ~15) + n * REQ_DTYPE.itemsize
    return n * REQ_DTYPE.itemsize


def expand_reqs(raw: np.ndarray, n: int, layout: int) -> np.ndarray:
    """[n] rhp_req_t records of a parsed batch from its raw reqs bytes in any layout
    (rhp_expand_reqs, include/rhp_host.h: dense records expanded)."""
    raw = np.ascontiguousarray(raw).view(np.uint8)
    if layout not in DENSE_LAYOUTS:
        return raw[: n * REQ_DTYPE.itemsize].view(REQ_DTYPE).copy()
    out = np.zeros(n, dtype=REQ_DTYPE)
    if n == 0:
        return out
    b = Batch(None, None, None, 0, n, 0, MODE_PHR, layout, None, None, None, None, 0, 0, None)
    rc = host().rhp_expand_reqs(ctypes.byref(b), _ptr(raw), _ptr(out))
    if rc != 0:
        raise RuntimeError(f"rhp_expand_reqs failed: {rc}")
    return out


def http_bytes(n: int, mode: int, layout: int) -> int:
    """bytes the batch's http buffer needs (rhp.h; RHP_COMPACT_HTTP_BYTES for the compact layout)"""
    if mode != MODE_HTTP:
        return HTTP_DTYPE.itemsize
    if layout in (LAYOUT_COMPACT, LAYOUT_DENSE):   # compact http records and their wide area
        return ((n * 8 + 15) & ~15) + n * HTTP_DTYPE.itemsize
    return n * HTTP_DTYPE.itemsize


def expand_http(reqs: np.ndarray, raw: np.ndarray, n: int, layout: int) -> np.ndarray:
    """[n] rhp_http_t records of a parsed http batch from its raw http bytes in any
    layout (rhp_expand_http, include/rhp_host.h: compact records expanded)."""
    raw = np.ascontiguousarray(raw).view(np.uint8)
    if layout not in (LAYOUT_COMPACT, LAYOUT_DENSE):
        return raw[: n * HTTP_DTYPE.itemsize].view(HTTP_DTYPE).copy()
    out = np.zeros(n, dtype=HTTP_DTYPE)
    if n == 0:
        return out
    reqs = np.ascontiguousarray(reqs)
    b = Batch(None, None, None, 0, n, 0, MODE_HTTP, layout, None, None, None, None, 0, 0, None)
    rc = host().rhp_expand_http(ctypes.byref(b), _ptr(reqs), _ptr(raw), _ptr(out))
    if rc != 0:
        raise RuntimeError(f"rhp_expand_http failed: {rc}")
    return out


def expand_records(reqs: np.ndarray, raw: np.ndarray, n: int, max_headers: int, layout: int) -> np.ndarray:
    """[n, max_headers] rhp_hdr_t records of a parsed batch from its raw hdrs bytes
    in any layout (rhp_expand_records, include/rhp_host.h): records of requests
    with ret <= 0 and past num_headers are zero."""
    out = np.zeros((n, max_headers), dtype=HDR_DTYPE)
    if n == 0 or max_headers == 0:
        return out
    reqs = np.ascontiguousarray(reqs)
    raw = np.ascontiguousarray(raw).view(np.uint8)
    b = Batch(None, None, None, 0, n, max_headers, MODE_PHR, layout, None, None, None, None, 0, 0, None)
    rc = host().rhp_expand_records(ctypes.byref(b), _ptr(reqs), _ptr(raw), _ptr(out))
    if rc != 0:
        raise RuntimeError(f"rhp_expand_records failed: {rc}")
    return out


def hdr_view(flat: np.ndarray, n: int, max_headers: int, layout: int) -> np.ndarray:
    """The [n, max_headers] view of a batch's record array in either layout (include/rhp.h)."""
    if layout == LAYOUT_HEADER_MAJOR:
        return flat[: n * max_headers].reshape(max_headers, n).T
    return flat[: n * max_headers].reshape(n, max_headers)


def _host_batch(buf, off, max_headers, mode, layout=LAYOUT_REQUEST_MAJOR, last_len=None, flags=0):
    n = len(off) - 1
    raw_reqs = np.zeros(max(reqs_bytes(n, layout), 8), dtype=np.uint8)
    reqs = raw_reqs[: n * REQ_DTYPE.itemsize].view(REQ_DTYPE)   # (dense: expanded by _host_done)
    raw = np.zeros(max(hdrs_bytes(n, max_headers, layout), 8), dtype=np.uint8)
    raw_http = np.zeros(max(http_bytes(n, mode, layout), 8), dtype=np.uint8)
    rw = buf.copy()
    b = Batch(_ptr(rw), _ptr(rw), _ptr(off), rw.size, n, max_headers, mode, layout, _ptr(raw_reqs), _ptr(raw),
              _ptr(raw_http), 0, flags, 0, _ptr(last_len) if last_len is not None else None)
    hv = None if layout in LENGTH_LAYOUTS else hdr_view(raw.view(HDR_DTYPE), n, max_headers, layout)
    res = Result(reqs, hv, None, rw)
    res.raw_reqs = raw_reqs
    res.raw_hdrs = raw   # the compact layout's records are expanded once the parse has run (_host_done)
    res.raw_http = raw_http if mode == MODE_HTTP else None
    return b, res


def _host_done(res: Result, n: int, max_headers: int, layout: int) -> Result:
    if layout in DENSE_LAYOUTS:
        res.reqs = expand_reqs(res.raw_reqs, n, layout)
    if layout in LENGTH_LAYOUTS:
        res.hdrs = expand_records(res.reqs, res.raw_hdrs, n, max_headers, layout)
    if res.raw_http is not None:
        res.http = expand_http(res.reqs, res.raw_http, n, layout)
    return res


def emulate(buf: np.ndarray, off: np.ndarray, max_headers: int = 16, mode: int = MODE_PHR,
            layout: int = LAYOUT_REQUEST_MAJOR, last_len: np.ndarray | None = None):
    """Run the kernel's DFA algorithm on the CPU (tests).  Returns (Result, stats[3]).
    last_len: optional u64[n], phr_parse_request's last_len per request (phr mode)."""
    if last_len is not None:
        last_len = np.ascontiguousarray(last_len, dtype=np.uint64)
    b, res = _host_batch(buf, off, max_headers, mode, layout, last_len)
    stats = np.zeros(3, dtype=np.uint64)
    rc = host().rhp_emu_parse_batch(ctypes.byref(b), _ptr(stats))
    if rc != 0:
        raise RuntimeError(f"rhp_emu_parse_batch failed: {rc}")
    return _host_done(res, len(off) - 1, max_headers, layout), stats


def parse_cpu_exact(buf: np.ndarray, off: np.ndarray, max_headers: int = 16, mode: int = MODE_PHR,
                    layout: int = LAYOUT_REQUEST_MAJOR):
    """The product's exact scalar parser on the host (rhp_scalar.h), e.g. for the reactor shim."""
    b, res = _host_batch(buf, off, max_headers, mode, layout)
    rc = host().rhp_cpu_parse_batch(ctypes.byref(b))
    if rc != 0:
        raise RuntimeError(f"rhp_cpu_parse_batch failed: {rc}")
    return _host_done(res, len(off) - 1, max_headers, layout)


class DeviceBatch:
    """A batch resident in HBM plus its output buffers (torch tensors as plumbing)."""

    def __init__(self, buf: np.ndarray, off: np.ndarray, max_headers: int = 16, mode: int = MODE_PHR,
                 device: str = "cuda", layout: int = LAYOUT_REQUEST_MAJOR, last_len: np.ndarray | None = None,
                 flags: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: the rhp product path runs on MI355X only")
        self.n = len(off) - 1
        self.max_headers = max_headers
        self.mode = mode
        self.layout = layout
        self.flags = flags
        self.bytes = torch.from_numpy(buf).to(device)
        self.offsets = torch.from_numpy(off.view(np.int64)).to(device)
        self.reqs = torch.zeros(max(reqs_bytes(self.n, layout), 8), dtype=torch.uint8, device=device)
        self.hdrs = torch.zeros(max(hdrs_bytes(self.n, max_headers, layout), 8), dtype=torch.uint8, device=device)
        self.http = torch.zeros(http_bytes(self.n, mode, layout), dtype=torch.uint8, device=device)
        self.work = torch.zeros(RHP_WORK_WORDS, dtype=torch.int32, device=device)
        self.last_len = (torch.from_numpy(np.ascontiguousarray(last_len, dtype=np.uint64).view(np.int64)).to(device)
                         if last_len is not None else None)

    def desc(self) -> Batch:
        return Batch(self.bytes.data_ptr(), self.bytes.data_ptr(), self.offsets.data_ptr(), self.bytes.numel(),
                     self.n, self.max_headers, self.mode, self.layout, self.reqs.data_ptr(), self.hdrs.data_ptr(),
                     self.http.data_ptr(), self.work.data_ptr(), self.flags, 0,
                     self.last_len.data_ptr() if self.last_len is not None else None)

    _runtime_checked = False   # one /proc/self/maps scan per process (it costs ~0.2 ms: not per launch)

    def launch(self, stream=None) -> None:
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        d = self.desc()
        if not DeviceBatch._runtime_checked:
            check_one_hip_runtime()   # the device buffers were allocated by torch's runtime by now
            DeviceBatch._runtime_checked = True
        rc = lib().rhp_parse_batch(ctypes.byref(d), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"rhp_parse_batch failed: {rc}")

    def result(self) -> Result:
        import torch
        torch.cuda.synchronize()
        raw_reqs = self.reqs.cpu().numpy()
        reqs = expand_reqs(raw_reqs, self.n, self.layout)
        raw = self.hdrs.cpu().numpy()
        hdrs = (expand_records(reqs, raw, self.n, self.max_headers, self.layout)
                if self.layout in LENGTH_LAYOUTS
                else hdr_view(raw.view(HDR_DTYPE), self.n, self.max_headers, self.layout))
        raw_http = self.http.cpu().numpy() if self.mode == MODE_HTTP else None
        http = expand_http(reqs, raw_http, self.n, self.layout) if self.mode == MODE_HTTP else None
        out = self.bytes.cpu().numpy() if self.mode == MODE_HTTP else None
        return Result(reqs, hdrs, http, out, raw, raw_http, raw_reqs)


def parse_batch(buf: np.ndarray, off: np.ndarray, max_headers: int = 16, mode: int = MODE_PHR,
                impl: int = IMPL_DFA, layout: int = LAYOUT_REQUEST_MAJOR, last_len: np.ndarray | None = None) -> Result:
    """Parse a host batch on the GPU (copies in, one launch, copies out)."""
    lib().rhp_set_impl(impl)
    try:
        db = DeviceBatch(buf, off, max_headers, mode, layout=layout, last_len=last_len)
        db.launch()
        return db.result()
    finally:
        lib().rhp_set_impl(IMPL_DFA)


def pack_dense_cpu(res: Result, n: int, max_headers: int):
    """rhp_cpu_pack_dense over the request-major http records of `res`: (dreq
    u8[8n], hc u8[8n], lens16 u16[max_headers * n]) -- what rhp_pack_dense makes
    on the device (include/rhp.h), the reactor's copy-back."""
    reqs = np.ascontiguousarray(res.raw_reqs[: n * REQ_DTYPE.itemsize]) if res.raw_reqs is not None \
        else np.ascontiguousarray(res.reqs).view(np.uint8)
    hdrs = np.ascontiguousarray(res.raw_hdrs)
    http = np.ascontiguousarray(res.raw_http)
    b = Batch(None, None, None, 0, n, max_headers, MODE_HTTP, LAYOUT_REQUEST_MAJOR, _ptr(reqs), _ptr(hdrs),
              _ptr(http), 0, 0, 0, None)
    dreq = np.zeros(max(8 * n, 8), dtype=np.uint8)
    hc = np.zeros(max(8 * n, 8), dtype=np.uint8)
    lens = np.zeros(max(max_headers * n, 1), dtype=np.uint16)
    rc = host().rhp_cpu_pack_dense(ctypes.byref(b), _ptr(dreq), _ptr(hc), _ptr(lens))
    if rc != 0:
        raise RuntimeError(f"rhp_cpu_pack_dense failed: {rc}")
    return dreq[: 8 * n], hc[: 8 * n], lens[: max_headers * n]


# ---------------------------------------------------------------------------
# Pipelined input (rhp.h rhp_fixup_sessions; the reference's server_session_read
# loop, /root/reference/src/reactor/server.c:37-65): a session's bytes split at
# every empty line into pieces, parsed speculatively, then walked in order.

def split_pieces(data: bytes):
    """Piece lengths of one session's input: a cut after every empty line (LF LF
    or LF CR LF, where a header section can end) and at the end."""
    cuts, n = [], len(data)
    p = data.find(b"\n")
    while p != -1:
        q = p + 1
        if q < n and data[q] == 10:
            cuts.append(q + 1)
        elif q + 1 < n and data[q] == 13 and data[q + 1] == 10:
            cuts.append(q + 2)
        p = data.find(b"\n", p + 1)
    out, at = [], 0
    for c in cuts:
        if c > at and c < n:
            out.append(c - at)
            at = c
    if at < n or not out:
        out.append(n - at)
    return out


def pack_sessions(sessions, split=True):
    """(buf, piece offsets, rhp_session_t array, session byte starts) for a list
    of session inputs packed back to back (split=False: one piece per session;
    a callable: data -> piece lengths, any split of the input)."""
    pieces, sess, starts, at = [], [], [], 0
    for data in sessions:
        lo = len(pieces)
        starts.append(at)
        for ln in (split(data) if callable(split) else split_pieces(data) if split else [len(data)]):
            pieces.append((at, ln))
            at += ln
        sess.append((lo, len(pieces)))
    off = np.zeros(len(pieces) + 1, dtype=np.uint64)
    for i, (a, ln) in enumerate(pieces):
        off[i] = a
    off[len(pieces)] = at
    buf = np.zeros(at + RHP_PAD, dtype=np.uint8)
    if at:
        buf[:at] = np.frombuffer(b"".join(sessions), dtype=np.uint8)
    ss = np.zeros(len(sess), dtype=SESSION_DTYPE)
    for i, (lo, hi) in enumerate(sess):
        ss[i] = (lo, hi)
    return buf, off, ss, np.array(starts, dtype=np.uint64)


def fixup_cpu(buf, off, sessions, max_headers: int = 16, emulate_dfa: bool = False, layout: int = LAYOUT_REQUEST_MAJOR):
    """Speculative http batch (host exact parser, or the kernel's DFA emulation)
    + rhp_cpu_fixup_sessions.  Returns (Result, session results, req_start)."""
    b, res = _host_batch(buf, off, max_headers, MODE_HTTP, layout, None, BATCH_SPECULATIVE)
    if emulate_dfa:
        rc = host().rhp_emu_parse_batch(ctypes.byref(b), None)
    else:
        rc = host().rhp_cpu_parse_batch(ctypes.byref(b))
    if rc != 0:
        raise RuntimeError(f"host parse failed: {rc}")
    out = np.zeros(len(sessions), dtype=SESSION_RESULT_DTYPE)
    starts = np.zeros(max(len(off) - 1, 1), dtype=np.uint64)
    rc = host().rhp_cpu_fixup_sessions(ctypes.byref(b), _ptr(sessions), len(sessions), _ptr(out), _ptr(starts))
    if rc != 0:
        raise RuntimeError(f"rhp_cpu_fixup_sessions failed: {rc}")
    return _host_done(res, len(off) - 1, max_headers, layout), out, starts


def fixup_gpu(buf, off, sessions, max_headers: int = 16, impl: int = IMPL_DFA, layout: int = LAYOUT_REQUEST_MAJOR):
    """Speculative http batch on the GPU + rhp_fixup_sessions, one stream."""
    import torch
    lib().rhp_set_impl(impl)
    try:
        db = DeviceBatch(buf, off, max_headers, MODE_HTTP, layout=layout, flags=BATCH_SPECULATIVE)
        db.launch()
        ds = torch.from_numpy(sessions.view(np.uint8).copy()).to("cuda")
        dres = torch.zeros(len(sessions) * SESSION_RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(max(db.n, 1) * 8, dtype=torch.uint8, device="cuda")
        d = db.desc()
        rc = lib().rhp_fixup_sessions(ctypes.byref(d), ctypes.c_void_p(ds.data_ptr()), len(sessions),
                                      ctypes.c_void_p(dres.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(f"rhp_fixup_sessions failed: {rc}")
        res = db.result()
        return res, dres.cpu().numpy().view(SESSION_RESULT_DTYPE), dst.cpu().numpy().view(np.uint64)
    finally:
        lib().rhp_set_impl(IMPL_DFA)


# ---------------------------------------------------------------------------
# Batched response serialization: http_write_response (src/reactor/http.c:286-297)
# for n responses on the device (rhp_writer.hip).  A batch is an arena of bytes
# plus rhp_resp_t records (n x 8 u32: status off,len, type off,len, body off,len,
# fields_first, fields_count) and rhp_resp_field_t records (m x 4 u32).

RESP_STATUS = (b"200 OK", b"404 Not Found", b"500 Internal Server Error", b"204 No Content",
               b"101 Switching Protocols")
RESP_TYPES = (b"text/plain", b"application/json", b"text/html; charset=UTF-8")
RESP_FIELD_NAMES = (b"Cookie", b"Set-Cookie", b"X-Request-Id", b"Cache-Control")
DEFAULT_DATE = b"Wed, 16 Aug 2023 10:29:23 GMT"


def make_responses(n: int, seed: int, kind: str = "mixed"):
    """Synthetic response batch (arena, resps, fields).  kind "plaintext": every
    response is the TechEmpower plaintext reply (200 OK, text/plain,
    "Hello, World!"); "mixed": seeded statuses/types, 0-3 extra fields, body
    lengths 0-2000 B with 1 % up to 100 kB (all digit counts of Content-Length)."""
    rng = np.random.default_rng(seed)
    parts, pos = [], 0

    def add(b: bytes):
        nonlocal pos
        parts.append(b)
        pos += len(b)
        return pos - len(b), len(b)

    st = [add(x) for x in RESP_STATUS]
    ty = [add(x) for x in RESP_TYPES]
    nm = [add(x) for x in RESP_FIELD_NAMES]
    resps = np.zeros((n, 8), dtype=np.uint32)
    fields = []
    if kind == "plaintext":
        body = add(b"Hello, World!")
        resps[:] = [st[0][0], st[0][1], ty[0][0], ty[0][1], body[0], body[1], 0, 0]
    else:
        pool = rng.integers(0x20, 0x7F, size=1 << 17, dtype=np.uint8).tobytes()
        pool_off, _ = add(pool)
        for i in range(n):
            s_, t_ = st[int(rng.integers(len(st)))], ty[int(rng.integers(len(ty)))]
            blen = int(rng.integers(0, 100001)) if rng.random() < 0.01 else int(rng.integers(0, 2001))
            bo = pool_off + int(rng.integers(0, len(pool) - blen + 1))
            nf = int(rng.integers(0, 4))
            first = len(fields)
            for _ in range(nf):
                vlen = int(rng.integers(0, 48))
                fields.append([*nm[int(rng.integers(len(nm)))], pool_off + int(rng.integers(0, 4096)), vlen])
            resps[i] = [s_[0], s_[1], t_[0], t_[1], bo, blen, first, nf]
    arena = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    f = np.array(fields, dtype=np.uint32).reshape(-1, 4) if fields else np.zeros((0, 4), dtype=np.uint32)
    return arena, resps, f


class DeviceResponses:
    """A response batch resident in HBM and its output (torch tensors as plumbing)."""

    def __init__(self, arena: np.ndarray, resps: np.ndarray, fields: np.ndarray, date: bytes = DEFAULT_DATE,
                 out_size: int | None = None, device: str = "cuda"):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: the rhp product path runs on MI355X only")
        self.n = len(resps)
        self.date = bytes(date)
        self.arena = torch.from_numpy(np.ascontiguousarray(arena, dtype=np.uint8)).to(device)
        self.resps = torch.from_numpy(np.ascontiguousarray(resps, dtype=np.uint32).view(np.int32)).to(device)
        fl = np.ascontiguousarray(fields, dtype=np.uint32).reshape(-1, 4)
        self.fields = torch.from_numpy(fl.view(np.int32)).to(device) if len(fl) else None
        self.out_off = torch.zeros(self.n + 1, dtype=torch.int64, device=device)
        if out_size is None:   # exact size from the host copy of the records
            r = np.asarray(resps, dtype=np.uint64).reshape(-1, 8)
            extra = 0
            if len(fl):
                fl64 = fl.astype(np.uint64)
                per = fl64[:, 1] + fl64[:, 3] + 4
                extra = int(sum(int(per[a:a + c].sum()) for a, c in zip(r[:, 6], r[:, 7]) if c))
            digits = np.array([len(str(int(v))) for v in r[:, 5]], dtype=np.uint64)
            out_size = int((95 + r[:, 1] + r[:, 3] + r[:, 5] + digits).sum()) + extra
        self.out = torch.zeros(max(out_size, 1), dtype=torch.uint8, device=device)
        self.out_size = out_size
        self.work = torch.zeros((self.n + 4095) // 4096 + 1, dtype=torch.int64, device=device)

    def desc(self) -> RespBatch:
        return RespBatch(self.arena.data_ptr(), self.resps.data_ptr(),
                         self.fields.data_ptr() if self.fields is not None else None, self.n, len(self.date),
                         self.date, self.out_off.data_ptr(), self.out.data_ptr(), self.out_size,
                         self.work.data_ptr())

    def launch(self, stream=None) -> None:
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        d = self.desc()
        rc = lib().rhp_write_responses(ctypes.byref(d), ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"rhp_write_responses failed: {rc}")

    def result(self):
        import torch
        torch.cuda.synchronize()
        off = self.out_off.cpu().numpy().view(np.uint64)
        return self.out.cpu().numpy()[: int(off[-1])], off


def write_responses(arena: np.ndarray, resps: np.ndarray, fields: np.ndarray, date: bytes = DEFAULT_DATE):
    """Serialize a host response batch on the GPU (copies in, one call, copies out):
    returns (bytes, offsets[n + 1])."""
    d = DeviceResponses(arena, resps, fields, date)
    d.launch()
    return d.result()
