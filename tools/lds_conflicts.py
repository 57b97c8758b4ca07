"""Offline model of the walk's LDS bank conflicts: the three
ds_read_u8 lookups of every pair step -- class row of b1, code of (b0, b1), the
dependent state read -- for the 64 lanes of a wave walking consecutive requests of
a config, with the pair table the kernel loads (rhp_test_table2).  LDS model of
MI355X_MICROARCH.md: a ds_read_b32-class access is two 32-lane groups, bank
(a / 4) mod 32, one cycle per distinct dword on the busiest bank.  Prints the
LDS cycles per wave-instruction of each lookup (2.0 = conflict free) and the
conflict fraction (extra / all cycles, as SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).

usage: python tools/lds_conflicts.py [config] [waves]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libreactorng_amd as rhp  # noqa: E402

S_SLOW, S_PRE = 2, 3   # rhp_dfa.h State


def table():
    h = rhp.host()
    h.rhp_test_table2.restype = ctypes.c_uint32
    meta = (ctypes.c_uint32 * 6)()
    n = h.rhp_test_table2(None, meta)
    t = np.zeros(n, dtype=np.uint8)
    h.rhp_test_table2(t.ctypes.data_as(ctypes.c_void_p), meta)
    return t, list(meta)


def cycles(addr):
    """LDS cycles of one wave-instruction (64 byte addresses)"""
    tot = 0
    for g in (addr[:32], addr[32:]):
        dw = np.unique(g >> 2)
        tot += int(np.bincount(dw % 32, minlength=32).max())
    return tot


def main():
    cfg = {"get256": rhp.GEN_GET256, "zipf": rhp.GEN_ZIPF, "post": rhp.GEN_POST1K}[sys.argv[1] if len(sys.argv) > 1 else "get256"]
    waves = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    T, meta = table()
    stride, crr = meta[1], meta[2]
    buf, off = rhp.generate(cfg, 64 * waves, 7)
    c1row, c16row = meta[3], meta[5]
    acc = np.zeros(3)
    acc2 = np.zeros(2)   # code form 2: class(b1), class(b0) * 16
    steps = 0
    for w in range(waves):
        req = np.arange(64 * w, 64 * w + 64)
        # the kernel's first windows: the 128-B line holding the request (phr mode), its
        # dword (http mode); the bytes before the request read as 0 and walk in S_PRE
        lead_mask = np.uint64(3 if cfg == rhp.GEN_POST1K else 127)
        s4 = (off[req] & ~lead_mask).astype(np.int64)
        lead = (off[req] & lead_mask).astype(np.int64)
        first = buf[off[req].astype(np.int64)]
        ctlx = ((first < 0x20) & (first != 9) & (first != 10) & (first != 13)) | (first == 0x7f)
        st = np.where(ctlx, 4 * S_SLOW, 4 * S_PRE).astype(np.int64)
        for p in range(128):   # two 128-B windows per lane
            b0 = np.where(2 * p < lead, 0, buf[s4 + 2 * p]).astype(np.int64)
            b1 = np.where(2 * p + 1 < lead, 0, buf[s4 + 2 * p + 1]).astype(np.int64)
            a_r = crr * 256 + b1
            r = T[a_r].astype(np.int64)
            a_c = r * 256 + b0
            c = T[a_c].astype(np.int64)
            a_s = st * stride + c
            acc += [cycles(a_r), cycles(a_c), cycles(a_s)]
            acc2 += [cycles(c1row * 256 + b1), cycles(c16row * 256 + b0)]
            st = T[a_s].astype(np.int64)
            steps += 1
    per = acc / steps
    print(f"row stride {stride}: LDS cycles per wave-instruction (2.0 = no conflict): "
          f"class row {per[0]:.2f}, code {per[1]:.2f}, state {per[2]:.2f}; "
          f"conflict fraction of the walk's lookups {(per.sum() - 6) / per.sum():.3f}")
    per2 = acc2 / steps
    print(f"code form 2 (class(b1) | class(b0) * 16): class {per2[0]:.2f}, class*16 {per2[1]:.2f}, state {per[2]:.2f}; "
          f"conflict fraction {(per2.sum() + per[2] - 6) / (per2.sum() + per[2]):.3f}")


if __name__ == "__main__":
    main()
