"""The libreactor surface (include/reactor.h, libreactorng_amd/libreactor.so):
the reference's example/server.c links against it unchanged, the http module
meets the reference's test/http.c expectations, and the HTTP server serves the
reference's test/server.c cases, BASELINE config 1 (16 pipelined 128-byte GETs)
and a pipelined many-connection load -- with the host parser on CPU and with
the MI355X batch parser on the GPU."""
import json
import os
import re
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "libreactorng_amd")
BIN = os.path.join(LIB, "bin")
REF_EXAMPLE = "/root/reference/example/server.c"


def _vectors(tmp_path):
    """tests/golden/http_request_tests.json (test/http.c:21-119) as the binary fixture http_test reads."""
    v = json.load(open(os.path.join(ROOT, "tests", "golden", "http_request_tests.json")))["vectors"]
    path = tmp_path / "vectors.bin"
    with open(path, "wb") as f:
        for x in v:
            b = x["request"].encode("latin-1")
            f.write(struct.pack("<I", len(b)) + b + struct.pack("<iI", x["result"], x["remaining"]))
    return str(path)


def _run(args, parser, timeout=120):
    env = dict(os.environ, RHP_REACTOR_PARSER=parser)
    p = subprocess.run(args, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def test_reactor_exports_every_declared_function():
    text = open(os.path.join(ROOT, "include", "reactor.h")).read()
    decl = set(re.findall(r"^(?!typedef)[a-z_0-9]+\s*\*?\s*([a-z_0-9]+)\s*\(", text, re.M))
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(LIB, "libreactor.so")], text=True)
    have = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert not sorted(decl - have)


@pytest.mark.skipif(not os.path.exists(REF_EXAMPLE), reason="reference checkout not present (dev container only)")
def test_reference_example_server_links_unchanged(tmp_path):
    """example/server.c of the reference, compiled and linked as it is."""
    exe = tmp_path / "server"
    subprocess.check_call(["gcc", "-std=gnu2x", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), REF_EXAMPLE,
                           "-o", str(exe), "-L", LIB, "-lreactor", f"-Wl,-rpath,{LIB}"])
    undefined = subprocess.check_output(["nm", "-u", str(exe)], text=True)
    used = {s for s in re.findall(r"U (\w+)", undefined) if not s.startswith("__")}
    assert {"reactor_construct", "reactor_loop", "reactor_destruct", "server_construct", "server_open",
            "server_plain", "string"} <= used


def test_http_module_reference_vectors(tmp_path):
    out = _run([os.path.join(BIN, "http_test"), _vectors(tmp_path)], "host")
    assert "read_request: 21 vectors" in out and "OK (0 failures)" in out


def test_server_cases_host_parser():
    out = _run([os.path.join(BIN, "server_test"), "16", "32"], "host")
    assert "parser: host" in out and "OK (0 failures)" in out
    assert "config1 16 pipelined   responses 16  callbacks 16" in out


@pytest.mark.parametrize("writer", ["host", "host-batch"])
def test_server_cases_host_async_parser(writer, monkeypatch):
    """Asynchronous rounds (batch.c "host-async": the gpu mode's slots and
    eventfd completion, parsed on a worker thread), replies written at once or
    batched per round: the same cases."""
    monkeypatch.setenv("RHP_REACTOR_WRITER", writer)
    out = _run([os.path.join(BIN, "server_test"), "32", "64"], "host-async")
    assert "parser: host-async" in out and "OK (0 failures)" in out
    assert "config1 16 pipelined   responses 16  callbacks 16" in out


def _burst(parser, conns=64, pipelined=64, reps=5, writer="host"):
    """burst_test: conns x pipelined requests land before the loop starts, so
    rounds hold conns x pipelined requests; req/s per burst (the first burst,
    which pays first-use costs, is dropped)."""
    env = dict(os.environ, RHP_REACTOR_PARSER=parser, RHP_REACTOR_STATS="1", RHP_REACTOR_WRITER=writer)
    p = subprocess.run([os.path.join(BIN, "burst_test"), str(conns), str(pipelined), str(reps)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "OK (0 failures)" in p.stdout, p.stdout + p.stderr
    rates = [float(x) for x in re.findall(r"\(([0-9.]+) req/s\)", p.stdout)]
    per_round = float(re.search(r"\(([0-9.]+) per round\)", p.stderr).group(1))
    return sorted(rates[1:])[len(rates[1:]) // 2], per_round, p.stdout + p.stderr


@pytest.mark.parametrize("parser", ["host", "host-async"])
def test_burst_rounds_host_parsers(parser):
    rate, per_round, out = _burst(parser, reps=3)
    assert per_round >= 4000, out


@pytest.mark.gpu
def test_burst_rounds_gpu_vs_host():
    """4096-request rounds (64 connections x 64 pipelined): the server with the
    MI355X parser (asynchronous rounds) against the host parser, same process
    layout; the numbers are printed (DESIGN.md §7 records a run)."""
    # two interleaved runs of each (gpu, host, gpu, host): a shared box's load
    # moves single runs by 20-30 %; each side keeps its better median
    runs = [(_burst("gpu", reps=9), _burst("host", reps=9)) for _ in range(2)]
    (gpu, gpu_round, out_g), (host, host_round, out_h) = (max((r[0] for r in runs), key=lambda x: x[0]),
                                                          max((r[1] for r in runs), key=lambda x: x[0]))
    gpu_w, _, out_w = _burst("gpu", writer="gpu", reps=9)
    print(f"burst req/s: gpu {gpu:.0f} ({gpu_round:.0f} requests/round), gpu parser + gpu writer {gpu_w:.0f}, "
          f"host {host:.0f} ({host_round:.0f})")
    print(out_g, out_w, out_h)
    assert gpu_round >= 4000 and host_round >= 4000
    # round completion by our own waiter thread blocked on the round's event
    # (RHP_REACTOR_COMPLETE=event, the default) rather than the HIP runtime's
    # host-function thread: 2.17 M req/s against the host parser's 2.19 M
    # (profiles/r03/reactor/); the parse is ~10 % of a burst's time.  Round 5
    # (registered slots, the wave-per-session fixup at 6 us instead of 187):
    # 2.07 M against 2.05 M, 16K-request rounds 2.80 M against 2.77 M and 65K
    # 3.33 M against 3.12 M (profiles/r05/reactor/).  Three runs of this test on one
    # box: 1.04, 0.96, 0.97 of the host parser (profiles/r05/reactor/burst_runs.txt);
    # the guard sits below that spread
    assert gpu >= 0.9 * host, (gpu, host)


@pytest.mark.gpu
@pytest.mark.parametrize("writer", ["host", "gpu"])
def test_server_cases_gpu_batch_parser(writer, monkeypatch):
    """The same cases with sessions parsed by rhp_parse_batch on the MI355X
    (asynchronous rounds), replies written at once or by rhp_write_responses
    once per round."""
    monkeypatch.setenv("RHP_REACTOR_WRITER", writer)
    out = _run([os.path.join(BIN, "server_test"), "64", "64"], "gpu")
    print(out)
    assert "parser: gpu" in out and "OK (0 failures)" in out
    assert "config1 16 pipelined   responses 16  callbacks 16" in out


@pytest.mark.parametrize("parser", ["host-async", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_server_first_round_after_late_completion(parser, monkeypatch):
    """the completion thread writes the eventfd before its queue
    entry leaves, so a round's completion is never still in flight when the
    queue looks empty (server_open's warm-up drains exactly its own rounds;
    a teardown drains all).  With every completion write held back 3 ms the
    first real rounds after server_open (the reference's cases first) and the
    load must still get their own replies."""
    monkeypatch.setenv("RHP_REACTOR_DELAY_COMPLETION_US", "3000")
    out = _run([os.path.join(BIN, "server_test"), "8", "16"], parser)
    assert f"parser: {parser}" in out and "OK (0 failures)" in out


def test_server_thread_exit_host_async():
    """A reactor thread serving with the asynchronous parser exits, three times
    over: its parser state (the worker thread, slots, eventfd) is torn down by
    the thread-exit hook, the worker joined before the state is freed."""
    out = _run([os.path.join(BIN, "thread_exit_test")], "host-async")
    assert "OK (0 failures)" in out and out.count("64 responses, exited") == 3


@pytest.mark.gpu
def test_server_thread_exit_gpu():
    """The same with the MI355X parser: the completion waiter thread, the
    round events, streams and pinned/device slots of an exiting reactor thread
    are released, and each new thread sets up (and warms up) its own."""
    out = _run([os.path.join(BIN, "thread_exit_test")], "gpu")
    assert "OK (0 failures)" in out and out.count("64 responses, exited") == 3


def test_reactor_host_code_asan_ubsan_clean(tmp_path):
    """libreactor.so, the host parser library and the two test programs built
    with -fsanitize=address,undefined (Makefile target `asan`): the reference's
    http vectors (buffer_append only, as test/http.c:134) and the server cases,
    long inputs included, run clean, leak check on."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(LIB, "csrc"), "asan"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    asan = os.path.join(LIB, "asan")
    for args, parser in (([os.path.join(asan, "http_test"), _vectors(tmp_path)], "host"),
                         ([os.path.join(asan, "server_test"), "8", "16"], "host"),
                         ([os.path.join(asan, "server_test"), "8", "16"], "host-async"),
                         ([os.path.join(asan, "thread_exit_test")], "host-async")):
        p = subprocess.run(args, env=dict(env, RHP_REACTOR_PARSER=parser), capture_output=True, text=True, timeout=300)
        assert p.returncode == 0 and "OK (0 failures)" in p.stdout, p.stdout + p.stderr
        assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr
