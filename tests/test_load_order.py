"""HIP runtime load order (VERDICT r5 'What's weak' 1b, 'Next' 6a).

librhp.so needs libamdhip64.so.7; torch's libc10_hip.so needs the unversioned
libamdhip64.so through its $ORIGIN rpath.  Loaded first, librhp.so would bring in
/opt/rocm's runtime and torch its own second copy (buffers of one are foreign to
the other: error 100 on the first launch).  libreactorng_amd.lib() preloads
torch's runtime by path, so either import order gives one runtime; a raw
CDLL of librhp.so before torch is detected and refused with the cause.  Each
case runs in a fresh child process (the load order is per process)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(code: str, timeout=300):
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests")))
    return p.returncode, p.stdout + p.stderr


def test_lib_before_torch_one_runtime():
    rc, out = child("import libreactorng_amd as r; r.lib(); import torch; rt = r.hip_runtimes(); "
                    "print('RUNTIMES', rt); assert len(rt) == 1, rt; r.check_one_hip_runtime()")
    assert rc == 0, out
    assert "torch/lib/libamdhip64.so" in out, out


def test_torch_before_lib_one_runtime():
    rc, out = child("import torch, libreactorng_amd as r; r.lib(); rt = r.hip_runtimes(); "
                    "assert len(rt) == 1, rt")
    assert rc == 0, out


def test_raw_cdll_before_torch_is_refused():
    rc, out = child("import ctypes, libreactorng_amd as r; ctypes.CDLL(r.LIBRHP); import torch\n"
                    "try:\n    r.check_one_hip_runtime()\nexcept RuntimeError as e:\n    print('REFUSED', e)")
    assert rc == 0 and "REFUSED two HIP runtimes" in out, out


@pytest.mark.gpu
def test_lib_before_torch_parses_on_gpu():
    """librhp.so loaded before torch, then a parse on the GPU against the oracle."""
    code = ("import libreactorng_amd as r; r.lib(); import torch\n"
            "from oracle_util import assert_same, canon, run_oracle, to_rhp\n"
            "buf, off = r.generate(r.GEN_GET256, 4096, 7)\n"
            "res = r.parse_batch(buf, off, 16, r.MODE_PHR, layout=r.LAYOUT_COMPACT)\n"
            "q, h, x, _ = run_oracle(buf, off, 16, r.MODE_PHR)\n"
            "assert_same(canon(res, r.MODE_PHR), to_rhp(q, h, x, r.MODE_PHR), buf, off, 'load order')\n"
            "print('PARSED', int((res.reqs['ret'] > 0).sum()), r.hip_runtimes())")
    rc, out = child(code, timeout=180)
    assert rc == 0 and "PARSED 4096" in out, out
