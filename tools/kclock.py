"""Diagnostic: shader clock of rhp_dfa_kernel under load (RHP_CLOCK build,
librhp_clock.so) and launch time per RHP_WAVES setting, for configs 2/3/5.
usage: RHP_LIB=libreactorng_amd/librhp_clock.so python tools/kclock.py"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libreactorng_amd as rhp
lib = rhp.lib()
lib.rhp_debug_clock.argtypes = [ctypes.c_void_p]
for cfg, seed, maxh, mode in ((rhp.GEN_GET256, 0x5EED0002, 16, 0), (rhp.GEN_ZIPF, 0x5EED0003, 32, 0),
                              (rhp.GEN_POST1K, 0x5EED0005, 16, 1)):
    buf, off = rhp.generate(cfg, 1 << 20, seed)
    dbs = [rhp.DeviceBatch(buf, off, maxh, mode) for _ in range(4)]
    for k in range(20):
        dbs[k % 4].launch()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for k in range(40):
        dbs[k % 4].launch()
    b.record()
    torch.cuda.synchronize()
    c = np.zeros(2, dtype=np.uint64)
    assert lib.rhp_debug_clock(c.ctypes.data) == 0
    print(f"config {cfg} waves {os.environ.get('RHP_WAVES', '16')}: {a.elapsed_time(b) / 40 * 1e3:.1f} us per launch, "
          f"block 0: {int(c[0])} ticks in {int(c[1]) / 100:.1f} us -> {c[0] / c[1] * 100:.0f} MHz", flush=True)
