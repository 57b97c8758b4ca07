"""Test-side access to the oracle (oracle/liboracle.so) and record comparison.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load the
oracle.  Canonical oracle records (oracle/rhp_oracle.h) are wide; `to_rhp`
converts them to the compact rhp.h layout so a whole batch compares with one
array equality.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

import libreactorng_amd as rhp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIBORACLE = os.path.join(ORACLE_DIR, "liboracle.so")
LIBREF = os.path.join(ORACLE_DIR, "_ref", "libref.so")

ORC_REQ = np.dtype([("ret", "<i4"), ("minor_version", "<i4"), ("num_headers", "<u4"), ("pad", "<u4"),
                    ("method_off", "<i8"), ("method_len", "<i8"), ("path_off", "<i8"), ("path_len", "<i8")])
ORC_HDR = np.dtype([("name_off", "<i8"), ("name_len", "<i8"), ("value_off", "<i8"), ("value_len", "<i8")])
ORC_HTTP = np.dtype([("result", "<i4"), ("body_kind", "<i4"), ("consumed", "<u8"), ("body_off", "<i8"),
                     ("body_len", "<u8")])

_orc = None
_ref = None


def oracle() -> ctypes.CDLL:
    global _orc
    if _orc is None:
        if not os.path.exists(LIBORACLE):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])
        _orc = ctypes.CDLL(LIBORACLE)
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        _orc.orc_phr_batch.argtypes = [vp, vp, u32, u32, vp, vp]
        _orc.orc_http_batch.argtypes = [vp, vp, u32, u32, vp, vp, vp]
        _orc.orc_phr_batch_mt.argtypes = [vp, vp, u32, u32, vp, vp, ctypes.c_int, ctypes.c_int]
        _orc.orc_phr_batch_mt.restype = ctypes.c_uint64
        _orc.orc_write_responses.argtypes = [vp, vp, vp, u32, ctypes.c_char_p, vp, vp]
        _orc.orc_write_responses.restype = ctypes.c_uint64
    return _orc


def reference():
    """The compiled reference (dev container only; None when /root/reference is absent)."""
    global _ref
    if _ref is None:
        if not os.path.exists(LIBREF):
            if not os.path.isdir("/root/reference"):
                return None
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "ref"])
        _ref = ctypes.CDLL(LIBREF)
        vp, u32 = ctypes.c_void_p, ctypes.c_uint32
        _ref.ref_phr_batch.argtypes = [vp, vp, u32, u32, vp, vp]
        _ref.ref_http_batch.argtypes = [vp, vp, u32, u32, vp, vp, vp]
        _ref.ref_write_responses.argtypes = [vp, vp, vp, u32, ctypes.c_char_p, vp, vp]
        _ref.ref_write_responses.restype = ctypes.c_uint64
    return _ref


def _run(libfn_phr, libfn_http, buf, off, max_headers, mode):
    n = len(off) - 1
    reqs = np.zeros(n, dtype=ORC_REQ)
    hdrs = np.zeros((n, max(max_headers, 1)), dtype=ORC_HDR)
    http = np.zeros(n, dtype=ORC_HTTP)
    rw = buf.copy()
    if mode == rhp.MODE_PHR:
        libfn_phr(rw.ctypes.data, off.ctypes.data, n, max_headers, reqs.ctypes.data, hdrs.ctypes.data)
    else:
        libfn_http(rw.ctypes.data, off.ctypes.data, n, max_headers, reqs.ctypes.data, hdrs.ctypes.data,
                   http.ctypes.data)
    return reqs, hdrs[:, :max_headers], http, rw


def run_oracle(buf, off, max_headers=16, mode=rhp.MODE_PHR):
    o = oracle()
    return _run(o.orc_phr_batch, o.orc_http_batch, buf, off, max_headers, mode)


def run_reference(buf, off, max_headers=16, mode=rhp.MODE_PHR):
    r = reference()
    return _run(r.ref_phr_batch, r.ref_http_batch, buf, off, max_headers, mode)


def to_rhp(reqs, hdrs, http, mode):
    """Wide oracle records -> canonical compact records (rhp.h layout)."""
    n = len(reqs)
    maxh = hdrs.shape[1]
    out = np.zeros(n, dtype=rhp.REQ_DTYPE)
    # a successful parse whose header section exceeds the u16 records is
    # RHP_RET_TOOLONG in the batch format (include/rhp.h)
    toolong = reqs["ret"] > rhp.RHP_MAX_LEN
    ok = (reqs["ret"] > 0) & ~toolong
    if mode == rhp.MODE_HTTP:
        ok &= http["result"] == 1
    out["ret"] = np.where(toolong, rhp.RHP_RET_TOOLONG, reqs["ret"])
    out["method_off"][ok] = reqs["method_off"][ok]
    out["method_len"][ok] = reqs["method_len"][ok]
    out["path_off"][ok] = reqs["path_off"][ok]
    out["path_len"][ok] = reqs["path_len"][ok]
    out["minor_version"] = -1
    out["minor_version"][ok] = reqs["minor_version"][ok]
    out["num_headers"][ok] = reqs["num_headers"][ok]
    h = np.zeros((n, maxh), dtype=rhp.HDR_DTYPE)
    if maxh:
        valid = ok[:, None] & (np.arange(maxh)[None, :] < reqs["num_headers"][:, None])
        name_off = np.where(hdrs["name_off"] < 0, rhp.RHP_NAME_NULL, hdrs["name_off"])
        for f, src in (("name_off", name_off), ("name_len", hdrs["name_len"]),
                       ("value_off", hdrs["value_off"]), ("value_len", hdrs["value_len"])):
            h[f] = np.where(valid, src, 0)
    x = None
    if mode == rhp.MODE_HTTP:
        x = np.zeros(n, dtype=rhp.HTTP_DTYPE)
        x["result"] = np.where(toolong, rhp.RHP_RET_TOOLONG, http["result"])
        one = (http["result"] == 1) & ~toolong
        x["body_kind"][one] = http["body_kind"][one]
        x["consumed"][one] = http["consumed"][one]
        x["body_len"][one] = http["body_len"][one]
        assert np.all(http["body_off"][one & (http["body_kind"] == 1)] ==
                      reqs["ret"][one & (http["body_kind"] == 1)])
        # bytes_out: a TOOLONG request's chunked body is not de-framed by the batch parser
    return out, h, x


def canon(res: rhp.Result, mode):
    """rhp.Result -> canonical records (fields unspecified by the reference zeroed):
    rhp.canonical, the one bench.py's parity check uses too."""
    return rhp.canonical(res, mode)


def assert_same(got, want, buf=None, off=None, label=""):
    """Compare canonical (reqs, hdrs, http) triples; report the first mismatch readably."""
    gr, gh, gx = got
    wr, wh, wx = want
    bad = gr != wr
    if gh.size:
        bad |= np.any(gh != wh, axis=1)
    if gx is not None:
        bad |= gx != wx
    if np.any(bad):
        i = int(np.flatnonzero(bad)[0])
        msg = [f"{label}: {int(bad.sum())} of {len(bad)} requests differ; first #{i}",
               f"  got  req {gr[i]}", f"  want req {wr[i]}"]
        if gh.size:
            msg += [f"  got  hdr {gh[i][: max(int(wr[i]['num_headers']), 1)]}",
                    f"  want hdr {wh[i][: max(int(wr[i]['num_headers']), 1)]}"]
        if gx is not None:
            msg += [f"  got  http {gx[i]}", f"  want http {wx[i]}"]
        if buf is not None:
            msg.append(f"  bytes {bytes(buf[int(off[i]):int(off[i + 1])])[:300]!r}")
        raise AssertionError("\n".join(msg))


def _write_responses(fn, arena, resps, fields, date):
    """http_write_response over a batch through fn (oracle or reference): (bytes, offsets)"""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    resps = np.ascontiguousarray(resps, dtype=np.uint32)
    fields = np.ascontiguousarray(fields, dtype=np.uint32).reshape(-1, 4)
    fp = fields.ctypes.data if len(fields) else None
    n = len(resps)
    off = np.zeros(n + 1, dtype=np.uint64)
    total = fn(arena.ctypes.data, resps.ctypes.data, fp, n, date, None, off.ctypes.data)
    out = np.zeros(max(int(total), 1), dtype=np.uint8)
    fn(arena.ctypes.data, resps.ctypes.data, fp, n, date, out.ctypes.data, off.ctypes.data)
    return out[: int(total)], off


def oracle_write_responses(arena, resps, fields, date=rhp.DEFAULT_DATE):
    return _write_responses(oracle().orc_write_responses, arena, resps, fields, date)


def reference_write_responses(arena, resps, fields, date=rhp.DEFAULT_DATE):
    ref = reference()
    assert ref is not None, "the compiled reference needs /root/reference"
    return _write_responses(ref.ref_write_responses, arena, resps, fields, date)
