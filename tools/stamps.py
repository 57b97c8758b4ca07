"""Diagnostic: per-section cycle breakdown of rhp_dfa_kernel (RHP_STAMPS build).

usage: python tools/stamps.py [config]   (needs libreactorng_amd/librhp_stamps.so)
Also reports the wall span of the launch in s_memtime ticks against the HIP-event
time of the same launch, i.e. the shader clock the kernel actually ran at.
"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["RHP_LIB"] = os.environ.get("RHP_STAMPS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "libreactorng_amd", "librhp_stamps.so"))
import torch
import libreactorng_amd as rhp
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else rhp.GEN_GET256
maxh = {rhp.GEN_ZIPF: 32}.get(cfg, 16)
mode = rhp.MODE_HTTP if cfg == rhp.GEN_POST1K else rhp.MODE_PHR
n = 1 << 20
buf, off = rhp.generate(cfg, n, 0x5EED0002)
db = rhp.DeviceBatch(buf, off, maxh, mode)
for _ in range(3):
    db.launch()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
db.launch()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b)
st = np.zeros(8192 * 8, dtype=np.uint64)
lib = rhp.lib()
lib.rhp_debug_stamps.argtypes = [ctypes.c_void_p]
assert lib.rhp_debug_stamps(st.ctypes.data) == 0
st = st.reshape(8192, 8)
used = st[:, 5] > 0
f = st.astype(np.float64)
tot = f[used, :5].sum(axis=0)
names = ["A top wait", "B decode+finalize", "C+D switch/refill", "E window issue", "F 64 steps"]
iters = f[used, 5].sum()
print(f"config {cfg}: waves {used.sum()}  iterations {iters:.0f}  cycles/iteration per wave:")
for k in range(5):
    print(f"  {names[k]:22s} {tot[k] / iters:9.1f}  ({100 * tot[k] / tot.sum():.1f}%)")
pre, whole = f[used, 6], f[used, 7]
print(f"  launch {ms * 1e3:.1f} us (HIP events); per wave: entry->loop {pre.mean():.0f}, entry->exit mean {whole.mean():.0f}"
      f" max {whole.max():.0f}, loop sections {tot.sum() / used.sum():.0f} (memtime ticks)")
# per-workgroup spread (waves g*W..g*W+W-1 form workgroup g; XCD = g % 8 under round-robin dispatch)
W = int(os.environ.get("RHP_WAVES", "16"))
ng = used.sum() // W
if ng:
    wg = whole[: ng * W].reshape(ng, W).max(axis=1)
    print(f"  per-workgroup entry->exit: min {wg.min():.0f} mean {wg.mean():.0f} max {wg.max():.0f}")
    xcd = np.array([wg[np.arange(ng) % 8 == x].mean() for x in range(8)])
    print("  mean per XCD (g % 8): " + " ".join(f"{v:.0f}" for v in xcd))
    slow = np.argsort(wg)[-8:]
    print("  slowest workgroups: " + " ".join(str(int(g)) for g in slow))
if ng and hasattr(lib, "rhp_debug_stamps_end"):
    se = np.zeros(8192, dtype=np.uint64)
    lib.rhp_debug_stamps_end.argtypes = [ctypes.c_void_p]
    assert lib.rhp_debug_stamps_end(se.ctypes.data) == 0
    end = se.astype(np.float64)[used]
    wg_loop = whole[: ng * W].reshape(ng, W).max(axis=1)
    wg_end = end[: ng * W].reshape(ng, W).max(axis=1)
    print(f"  per-workgroup loop end (last wave) mean {wg_loop.mean():.0f}, replay end mean {wg_end.mean():.0f} max {wg_end.max():.0f}"
          f"  -> replay {100 * (wg_end - wg_loop).mean() / wg_end.mean():.1f} % of the workgroup span")
if ng:
    per_idx = whole[: ng * W].reshape(ng, W)
    print("  mean entry->exit by wave index in workgroup: " + " ".join(f"{v / 1000:.0f}k" for v in per_idx.mean(axis=0)))
    its = f[used, 5][: ng * W].reshape(ng, W)
    print("  mean iterations by wave index: " + " ".join(f"{v:.1f}" for v in its.mean(axis=0)))
