"""Diagnostic: per-launch time of rhp_parse_batch on one stream (HIP events)
against back-to-back batches on S streams (batch k+1 starting on the CUs batch
k's tail frees), configs 2, 3, 5.  usage: python tools/pipeline_probe.py [S]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for key, steps in (("get256", 40), ("zipf", 12), ("post", 30)):
    cfg = bench.CONFIGS[key]
    r = bench.GpuRunner(cfg, 0, cfg["per_gpu"], 4, bench.LAYOUTS[cfg["layout"]], streams=S)
    for k in range(6):
        r.step(k)
    r.sync()
    wall1, kern = r.timed(steps)
    for k in range(6):
        r.step(k)
    walls = [r.timed_pipelined(steps) for _ in range(3)]
    ws = min(walls)
    print(f"{key:7s} one stream: kernel {kern * 1e3:7.1f} us, wall/step {wall1 / steps * 1e6:7.1f} us | "
          f"{S} streams: wall/step {ws / steps * 1e6:7.1f} us (runs {', '.join(f'{w / steps * 1e6:.1f}' for w in walls)})",
          flush=True)
