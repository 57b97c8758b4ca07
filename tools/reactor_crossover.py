"""Where the reactor's GPU parser passes the host parser.

tests/reactor/burst_test.c at round sizes of 4K, 16K and 64K requests (C
connections x P pipelined 128-B TFB GETs land before the loop starts, so a
round holds C x P requests), with RHP_REACTOR_PARSER=gpu and =host, a fresh
server per burst.  Per size and parser: the median requests/s over the bursts
after the first, the first burst's time (GPU setup now happens in server_open,
before the timed loop), and the parser's per-round submit-to-result time
(RHP_REACTOR_STATS).  Interleaved gpu, host, gpu, host so a shared box's drift
hits both.

usage: python tools/reactor_crossover.py [--reps 7] > profiles/.../crossover.txt
"""
import argparse
import os
import re
import statistics
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "libreactorng_amd", "bin", "burst_test")


def burst(parser, conns, per_conn, reps):
    env = dict(os.environ, RHP_REACTOR_PARSER=parser, RHP_REACTOR_STATS="1")
    p = subprocess.run([BIN, str(conns), str(per_conn), str(reps)], env=env, capture_output=True, text=True,
                       timeout=600)
    if p.returncode != 0 or "OK (0 failures)" not in p.stdout:
        raise RuntimeError(p.stdout + p.stderr)
    ms = [float(x) for x in re.findall(r"responses in ([0-9.]+) ms", p.stdout)]
    rates = [float(x) for x in re.findall(r"\(([0-9.]+) req/s\)", p.stdout)]
    per_round = re.search(r"\(([0-9.]+) per round\), ([0-9.]+) us per round", p.stderr)
    return dict(first_ms=ms[0], median_rate=statistics.median(rates[1:]), best_rate=max(rates[1:]),
                requests_per_round=float(per_round.group(1)) if per_round else None,
                us_per_round=float(per_round.group(2)) if per_round else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    sizes = [(64, 64), (128, 128), (256, 256)]
    print(f"{'round':>7} {'parser':>6} {'median req/s':>13} {'best req/s':>11} {'first burst ms':>15} "
          f"{'req/round':>10} {'us/round':>9}")
    for conns, per in sizes:
        res = {"gpu": [], "host": []}
        for _ in range(2):
            for parser in ("gpu", "host"):
                res[parser].append(burst(parser, conns, per, a.reps))
        for parser in ("gpu", "host"):
            r = max(res[parser], key=lambda x: x["median_rate"])
            print(f"{conns * per:>7} {parser:>6} {r['median_rate']:>13.0f} {r['best_rate']:>11.0f} "
                  f"{r['first_ms']:>15.3f} {r['requests_per_round'] or 0:>10.0f} {r['us_per_round'] or 0:>9.1f}",
                  flush=True)


if __name__ == "__main__":
    main()
