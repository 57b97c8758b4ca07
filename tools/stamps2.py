"""Diagnostic: per-section shader cycles of rhp_dfa_kernel (RHP_STAMPS build,
RHP_LIB=librhp_x_stamps.so) for configs 2, 3, 5 at bench's layouts."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libreactorng_amd as rhp
lib = rhp.lib()
lib.rhp_debug_stamps.argtypes = [ctypes.c_void_p]
names = ["A wait window", "C-E switch/refill/issue", "decode", "walk", "finalize/handover"]
for cfg, seed, maxh, mode, layout in ((rhp.GEN_GET256, 0x5EED0002, 16, 0, 1), (rhp.GEN_ZIPF, 0x5EED0003, 32, 0, 0),
                                      (rhp.GEN_POST1K, 0x5EED0005, 16, 1, 1)):
    buf, off = rhp.generate(cfg, 1 << 20, seed)
    dbs = [rhp.DeviceBatch(buf, off, maxh, mode, layout=layout) for _ in range(4)]
    for c in dbs[1:]:
        c.reqs, c.hdrs, c.http = dbs[0].reqs, dbs[0].hdrs, dbs[0].http
    for k in range(12):
        dbs[k % 4].launch()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    dbs[0].launch()
    b.record()
    torch.cuda.synchronize()
    st = np.zeros(8192 * 8, dtype=np.uint64)
    assert lib.rhp_debug_stamps(st.ctypes.data) == 0
    st = st.reshape(8192, 8).astype(np.float64)
    used = st[:, 5] > 0
    tot = st[used, :5].sum(axis=0)
    it = st[used, 5].sum()
    print(f"config {cfg}: {a.elapsed_time(b) * 1e3:.1f} us, waves {used.sum()}, iterations {it:.0f} "
          f"({it / used.sum():.1f} per wave), cycles per iteration per wave:")
    for k in range(5):
        print(f"   {names[k]:26s} {tot[k] / it:8.0f}  ({100 * tot[k] / tot.sum():.1f} %)")
    print(f"   per wave: {st[used, :5].sum(axis=1).mean():.0f} cycles in the loop", flush=True)
