"""Diagnostic: per-section shader cycles of rhp_dfa_kernel (RHP_STAMPS build,
RHP_LIB=librhp_x_stamps.so) for configs 2, 3, 5 at bench's layouts, and the
launch's timeline from the realtime marks (entry, loop start, loop end, exit;
100 MHz ticks)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libreactorng_amd as rhp
SLOTS = 24
lib = rhp.lib()
lib.rhp_debug_stamps.argtypes = [ctypes.c_void_p]
# section names: early-issue kernel (phr mode) / late-issue kernel (http mode)
names = ["A wait window / + framing finish", "C-E switch/refill/issue / C-D switch/refill",
         "decode / decode + finalize", "walk", "finalize/handover / issue"]
NREQ = int(os.environ.get("STAMPS_N", 1 << 20))
ONLY = os.environ.get("STAMPS_CFG")
for cfg, seed, maxh, mode, layout in ((rhp.GEN_GET256, 0x5EED0002, 16, 0, rhp.LAYOUT_COMPACT),
                                      (rhp.GEN_ZIPF, 0x5EED0003, 32, 0, 0),
                                      (rhp.GEN_POST1K, 0x5EED0005, 16, 1, rhp.LAYOUT_COMPACT), (rhp.GEN_CHUNKED, 0x5EED0006, 16, 1, 1)):
    if ONLY and str(cfg) not in ONLY.split(","):
        continue
    buf, off = rhp.generate(cfg, NREQ, seed)
    dbs = [rhp.DeviceBatch(buf, off, maxh, mode, layout=layout) for _ in range(4)]
    for c in dbs[1:]:
        c.reqs, c.hdrs, c.http = dbs[0].reqs, dbs[0].hdrs, dbs[0].http
    pristine = dbs[0].bytes.clone() if cfg == rhp.GEN_CHUNKED else None   # its launches de-frame in place
    for k in range(12):
        if pristine is not None:
            dbs[k % 4].bytes.copy_(pristine)
        dbs[k % 4].launch()
    torch.cuda.synchronize()
    if pristine is not None:
        dbs[0].bytes.copy_(pristine)
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    dbs[0].launch()
    b.record()
    torch.cuda.synchronize()
    st = np.zeros(8192 * SLOTS, dtype=np.uint64)
    assert lib.rhp_debug_stamps(st.ctypes.data) == 0
    st = st.reshape(8192, SLOTS).astype(np.float64)
    used = st[:, 5] > 0
    tot = st[used, :5].sum(axis=0)
    it = st[used, 5].sum()
    print(f"config {cfg}: {a.elapsed_time(b) * 1e3:.1f} us, waves {used.sum()}, iterations {it:.0f} "
          f"({it / used.sum():.1f} per wave), cycles per iteration per wave:")
    for k in range(5):
        print(f"   {names[k]:26s} {tot[k] / it:8.0f}  ({100 * tot[k] / tot.sum():.1f} %)")
    if st[used, 20].sum() > 0 and mode == 1:
        print(f"     (late form: section 2 = decode_window {st[used, 20].sum() / it:.0f} + frame_window "
              f"{st[used, 21].sum() / it:.0f} + decode_end/finalize)")
    elif st[used, 20].sum() > 0:
        print(f"     (early form, before section C-E: window reads + switch {st[used, 20].sum() / it:.0f}, "
              f"shuffles + refill {st[used, 21].sum() / it:.0f}; C-E is then the loads' issue)")
    loop = st[used, :5].sum(axis=1)
    print(f"   per wave: {loop.mean():.0f} cycles in the loop (min {loop.min():.0f}, max {loop.max():.0f})")
    rt = np.concatenate([st[used, 6:10], st[used, 14:15]], axis=1) * 10.0 / 1000.0   # us
    t0 = rt[:, 0].min()
    rt = rt - t0
    q = lambda v: f"{np.percentile(v, 0):6.1f} {np.percentile(v, 50):6.1f} {np.percentile(v, 99):6.1f} {v.max():6.1f}"
    print("   timeline us from the first entry (min / median / p99 / max):")
    print(f"     entry       {q(rt[:, 0])}")
    print(f"     loop start  {q(rt[:, 1])}   prologue {q(rt[:, 1] - rt[:, 0])}")
    ld = st[used, 19] * 10.0 / 1000.0 - t0
    print(f"     prologue loads landed {q(ld)}   entry->loads {q(ld - rt[:, 0])}   loads->loop start {q(rt[:, 1] - ld)}")
    print(f"     loop end    {q(rt[:, 2])}   loop     {q(rt[:, 2] - rt[:, 1])}")
    print(f"     exit        {q(rt[:, 3])}   barrier  {q(rt[:, 4] - rt[:, 2])}   replay {q(rt[:, 3] - rt[:, 4])}")
    # by wave slot in the workgroup (dispatch age): iterations and loop end
    idx = np.nonzero(used)[0] % 16
    its = st[used, 5]
    print("   by wave slot: iterations / loop end us (mean)")
    print("     " + " ".join(f"{its[idx == k].mean():5.1f}" for k in range(16)))
    print("     " + " ".join(f"{rt[idx == k, 2].mean():5.1f}" for k in range(16)))
    wg = np.nonzero(used)[0] // 16
    ends = np.array([rt[wg == g, 2].max() for g in np.unique(wg)])
    firsts = np.array([rt[wg == g, 2].min() for g in np.unique(wg)])
    nw_, ni_ = st[used, 10], st[used, 11]
    print("   by wave slot: lane occupancy (walked / (walked + idle))")
    print("     " + " ".join(f"{nw_[idx == k].sum() / (nw_[idx == k].sum() + ni_[idx == k].sum()):5.2f}" for k in range(16)))
    il, dry = st[used, 12], st[used, 13]
    print(f"   idle lane-iterations: {ni_.sum():.0f}, of them while the pool had requests {il.sum():.0f}; "
          f"iterations after the pool ran dry: {dry.mean():.1f} per wave (of {st[used, 5].mean():.1f})")
    rx = st[used, 15:19]
    print(f"   replay per wave: pass 1 (hint framing) {rx[:, 1].mean():.0f} cycles ({rx[:, 3].mean():.1f} requests framed), "
          f"pass 2 (listed scalar paths) {rx[:, 0].mean():.0f} cycles ({rx[:, 2].mean():.1f} requests)")
    if st[used, 22].sum() + st[used, 23].sum() > 0:
        print(f"     pass 2 parts per wave: validation + serial paths {st[used, 22].mean():.0f} cycles, "
              f"staged moves {st[used, 23].mean():.0f} cycles")
    print(f"   workgroups: last wave's loop end {q(ends)}; first wave's {q(firsts)}", flush=True)
    if (rt[:, 3] - rt[:, 4]).mean() > 50.0:   # a long replay (chunked): where its time goes
        ex_last = np.array([rt[wg == g, 3].max() for g in np.unique(wg)])
        ex_first = np.array([rt[wg == g, 3].min() for g in np.unique(wg)])
        print(f"   workgroups: last wave's exit {q(ex_last)}; first wave's exit {q(ex_first)}")
        print("   by wave slot: replay us (mean)")
        print("     " + " ".join(f"{(rt[idx == k, 3] - rt[idx == k, 4]).mean():5.0f}" for k in range(16)))
        ug = np.unique(wg)
        print("   by XCD (workgroup mod 8): last wave's exit us (mean)")
        print("     " + " ".join(f"{ex_last[(ug % 8) == x].mean():6.1f}" for x in range(8)), flush=True)
