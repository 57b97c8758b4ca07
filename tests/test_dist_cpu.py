"""CPU, world_size 2 over gloo: the N>1 bench path (contiguous request shards,
no data-path collective, max-over-ranks timing, summed algorithmic bytes)
reproduces the single-process result.  Each rank parses its shard with the CPU
emulation of the kernel (the GPU kernel itself is covered by the -m gpu tests)."""
import os
import socket
import tempfile

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import libreactorng_amd as rhp

N_TOTAL = 6000
SEED = 0x5EED0003


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard_range(N_TOTAL, rank, world)
    buf, off = rhp.generate(rhp.GEN_ZIPF, hi - lo, SEED, lo=lo)
    res, _ = rhp.emulate(buf, off, 32)
    np.save(os.path.join(outdir, f"ret{rank}.npy"), res.reqs["ret"])
    alg = torch.tensor([float(rhp.header_bytes(rhp.GEN_ZIPF, hi - lo, SEED, lo=lo))], dtype=torch.float64)
    dist.all_reduce(alg)
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        np.save(os.path.join(outdir, "agg.npy"), np.array([float(alg[0]), float(t[0])]))
    dist.barrier()
    dist.destroy_process_group()


def test_shards_partition_and_match_single_process():
    world = 2
    assert [bench.shard_range(10, r, 3) for r in range(3)] == [(0, 3), (3, 6), (6, 10)]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, start_method="spawn")
        rets = np.concatenate([np.load(os.path.join(d, f"ret{r}.npy")) for r in range(world)])
        alg, tmax = np.load(os.path.join(d, "agg.npy"))
    buf, off = rhp.generate(rhp.GEN_ZIPF, N_TOTAL, SEED)
    full, _ = rhp.emulate(buf, off, 32)
    assert np.array_equal(rets, full.reqs["ret"])
    assert alg == rhp.header_bytes(rhp.GEN_ZIPF, N_TOTAL, SEED)
    assert tmax == 1.5


def _bench(args, env=None):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=e, capture_output=True,
                       text=True, timeout=600)
    lines = [line for line in p.stdout.splitlines() if line.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 rank processes itself
    (gloo control plane, contiguous shards, max-over-ranks time, summed bytes);
    --device cpu runs the kernel's CPU emulation in place of the GPU."""
    rc, line, err = _bench(["--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1", "--no-cpu",
                            "--per-gpu", "32768"])
    assert rc == 0, err
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "shard2"
    assert line["config"]["global_requests"] == 65536 and line["config"]["requests_per_gpu"] == 32768
    assert line["config"]["ok_fraction"] == 1.0 and line["value"] > 0


def test_bench_rejects_world_size_mismatch():
    rc, line, _ = _bench(["--gpus", "4", "--device", "cpu", "--steps", "1", "--no-cpu", "--per-gpu", "1024"],
                         env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2 and line is None
