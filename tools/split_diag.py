import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
torch.cuda.set_device(0)
import libreactorng_amd as rhp
buf, off = rhp.generate(rhp.GEN_ZIPF, 1 << 20, 0x5EED0003)
L = np.diff(off.astype(np.int64))
for maxh in (32,):
    res = rhp.parse_batch(buf, off, maxh, rhp.MODE_PHR)
    ex = (res.reqs["flags"] & rhp.F_EXACT) != 0
    big = (L >= 2048) & (L <= 32768)
    print("maxh", maxh, "exact total", ex.sum(), "exact among split-size", (ex & big).sum(), "of", big.sum(),
          "exact among others", (ex & ~big).sum())
    idx = np.nonzero(ex & big)[0][:5]
    for i in idx:
        r = res.reqs[i]
        print(i, L[i], r["ret"], r["num_headers"], r["path_len"])
