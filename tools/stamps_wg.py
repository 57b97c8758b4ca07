"""Diagnostic (RHP_STAMPS build, RHP_LIB=librhp_x_stamps.so): config 3's workgroup
loop ends against each workgroup range's work -- its windows in all and its
longest request's windows -- to tell work imbalance across ranges from speed
differences (a range's end cannot come before its longest request's walk)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libreactorng_amd as rhp
SLOTS = 24
lib = rhp.lib()
lib.rhp_debug_stamps.argtypes = [ctypes.c_void_p]
n = 1 << 20
buf, off = rhp.generate(rhp.GEN_ZIPF, n, 0x5EED0003)
dbs = [rhp.DeviceBatch(buf, off, 32, 0, layout=0) for _ in range(4)]
for k in range(12):
    dbs[k % 4].launch()
torch.cuda.synchronize()
dbs[0].launch()
torch.cuda.synchronize()
st = np.zeros(8192 * SLOTS, dtype=np.uint64)
assert lib.rhp_debug_stamps(st.ctypes.data) == 0
st = st.reshape(8192, SLOTS).astype(np.float64)
used = st[:, 5] > 0
rt = st[:, 6:10] * 10.0 / 1000.0
t0 = rt[used, 0].min()
wg = np.nonzero(used)[0] // 16
G = wg.max() + 1
end = np.array([rt[np.nonzero(used)[0][wg == g], 2].max() - t0 for g in range(G)])
span = (n + G - 1) // G
L = np.diff(off).astype(np.int64)
lead = (off[:-1] % 128).astype(np.int64)
win = (L + lead + 127) // 128
tot = np.array([win[g * span:(g + 1) * span].sum() for g in range(G)])
mx = np.array([win[g * span:(g + 1) * span].max() for g in range(G)])
print(f"workgroups {G}, span {span}; loop end us: min {end.min():.1f} median {np.median(end):.1f} max {end.max():.1f}")
print(f"windows per range: min {tot.min()} median {np.median(tot):.0f} max {tot.max()}; longest request windows: "
      f"min {mx.min()} median {np.median(mx):.0f} max {mx.max()}")
print(f"correlation of loop end with the range's windows {np.corrcoef(end, tot)[0, 1]:.2f}, "
      f"with its longest request {np.corrcoef(end, mx)[0, 1]:.2f}")
xcd = np.arange(G) % 8
print("loop end by XCD (mean): " + " ".join(f"{end[xcd == x].mean():.1f}" for x in range(8)))
order = np.argsort(end)
print("slowest 8 ranges: end / windows / longest: " + "; ".join(f"{end[g]:.0f}/{tot[g]}/{mx[g]}" for g in order[-8:]))
print("fastest 8 ranges: end / windows / longest: " + "; ".join(f"{end[g]:.0f}/{tot[g]}/{mx[g]}" for g in order[:8]), flush=True)
