"""A large GPU fuzz run against the oracle (a one-off check beside the GPU suite's
60K-request fuzz): N fuzz requests (GEN_FUZZ phr, GEN_FUZZ_HTTP http) per seed,
every record layout (round 6: the dense ones too), the kernel's records against the oracle's and its
DFA / exact-path choice (flags) against the emulator's.  Prints one line per
case; exits 1 on the first mismatch.

usage: python tools/fuzz_gpu_big.py [n] [seeds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import libreactorng_amd as rhp  # noqa: E402
from oracle_util import assert_same, canon, run_oracle, to_rhp  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    total = 0
    for seed in range(seeds):
        for gen, mode in ((rhp.GEN_FUZZ, rhp.MODE_PHR), (rhp.GEN_FUZZ_HTTP, rhp.MODE_HTTP)):
            buf, off = rhp.generate(gen, n, 7100 + seed)
            for maxh in (0, 3, 16, 64):
                want = to_rhp(*run_oracle(buf, off, maxh, mode)[:3], mode)
                lays = [rhp.LAYOUT_REQUEST_MAJOR, rhp.LAYOUT_HEADER_MAJOR, rhp.LAYOUT_COMPACT, rhp.LAYOUT_DENSE]
                if mode == rhp.MODE_PHR:
                    lays.append(rhp.LAYOUT_DENSE_RM)   # (request-major dense: phr mode only)
                for layout in lays:
                    res = rhp.parse_batch(buf, off, maxh, mode, layout=layout)
                    assert_same(canon(res, mode), want, buf, off, f"fuzz seed {seed} mode {mode} maxh {maxh} layout {layout}")
                    emu, _ = rhp.emulate(buf, off, maxh, mode, layout)
                    same = np.array_equal(res.reqs["flags"] & (rhp.F_EXACT | rhp.F_WIDE),
                                          emu.reqs["flags"] & (rhp.F_EXACT | rhp.F_WIDE))
                    exact = int(((res.reqs["flags"] & rhp.F_EXACT) != 0).sum())
                    print(f"seed {seed} mode {mode} maxh {maxh:2d} layout {layout}: {len(off) - 1} requests match the oracle, "
                          f"exact path {exact}, flags as the emulator: {same}", flush=True)
                    if not same:
                        sys.exit(1)
                    total += len(off) - 1
    print(f"fuzz_gpu_big OK: {total} request parses")


if __name__ == "__main__":
    main()
