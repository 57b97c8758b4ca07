"""Where the chunked config's time goes: the same batch parsed with the bodies
de-framed in place (restored before each launch), validated only (the
speculative flag: no byte is written), and config 5's CL POSTs of the same
count for the DFA loop alone.  Kernel ms from HIP events."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libreactorng_amd as rhp  # noqa: E402


def timed(db, reps=5, pristine=None):
    ms = []
    for _ in range(reps):
        if pristine is not None:
            db.bytes.copy_(pristine)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        db.launch()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return min(ms), sorted(ms)[len(ms) // 2]


for n in [int(x) for x in (sys.argv[1:] or ["65536", "1048576"])]:
    buf, off = rhp.generate(rhp.GEN_CHUNKED, n, 0x5EED0006)
    db = rhp.DeviceBatch(buf, off, 16, rhp.MODE_HTTP, layout=rhp.LAYOUT_HEADER_MAJOR)
    pristine = db.bytes.clone()
    full = timed(db, pristine=pristine)
    spec = rhp.DeviceBatch(buf, off, 16, rhp.MODE_HTTP, layout=rhp.LAYOUT_HEADER_MAJOR, flags=rhp.BATCH_SPECULATIVE)
    val = timed(spec)
    pb, po = rhp.generate(rhp.GEN_POST1K, n, 0x5EED0005)
    post = timed(rhp.DeviceBatch(pb, po, 16, rhp.MODE_HTTP, layout=rhp.LAYOUT_HEADER_MAJOR))
    print(f"n={n}: chunked de-framed {full[0]:.3f}/{full[1]:.3f} ms, validated only {val[0]:.3f}/{val[1]:.3f} ms, "
          f"CL POST {post[0]:.3f}/{post[1]:.3f} ms (min/median)", flush=True)
