#!/bin/bash
# One GPU session of evidence for the committed kernel: the GPU test suite, the
# bench line, rocprofv3 kernel-trace summaries of configs 2/3/5 and PMC
# FETCH_SIZE / WRITE_SIZE passes (separate runs).  Every GPU step has its own
# time limit; steps are chained with && so a failure stops the session.
# STEPS=tests,bench,prof,pmc,sq,writer,smoke,ceil (default all but ceil); also
#   quick  the GPU tests whose names match TESTS_K (pytest -k)
#   lines  tools/ubench_lines (window line order vs bandwidth; built beforehand)
#   ab     tools/ab_libs.py over AB_LIBS ("tag=path ...") for each of AB_CONFIGS
#   stamps tools/stamps2.py on the RHP_STAMPS build (librhp_x_stamps.so) for STAMPS_CFG
#   reactor tools/reactor_timeline.sh and two tools/reactor_crossover.py runs
# (round 6: one script for every session; the per-session env is recorded in
# the profiles README that keeps its output)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-s}
STEPS=${STEPS:-tests,bench,prof,pmc,sq,writer,smoke}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
ok=0
step_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1 && echo TESTS_OK && tail -3 gpurun_out/pytest_${TAG}.log
}
step_bench() {
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
    && cat gpurun_out/bench_${TAG}.json
}
step_prof() {
  for c in get256 zipf post chunked; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_$c -o run \
      -- python3 bench.py --config $c --extra none --steps 30 --warmup 5 --streams 1 --no-cpu --no-e2e > gpurun_out/prof_${TAG}_$c.log 2>&1 \
      || return 1
    echo PROF_${c}_OK
  done
}
step_pmc() {
  for c in get256 zipf post chunked; do
    for k in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d gpurun_out/pmc_${TAG}_${c}_$k -o p \
        -- python3 bench.py --config $c --extra none --steps 6 --warmup 2 --no-cpu --no-e2e > gpurun_out/pmc_${TAG}_${c}_$k.log 2>&1 \
        || return 1
    done
    echo PMC_${c}_OK
  done
}
step_sq() {
  for c in ${SQ_CONFIGS:-get256 zipf post chunked}; do
    TAG=sq_${TAG}_$c CONFIG=$c bash tools/pmc_sq.sh > gpurun_out/sq_${TAG}_$c.txt 2>&1 || return 1
    echo SQ_${c}_OK
  done
}
step_writer() {
  timeout -k 10 120 python3 tools/bench_writer.py > gpurun_out/writer_${TAG}.json 2>&1 \
    && timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${TAG}_writer -o run \
      -- python3 tools/bench_writer.py > gpurun_out/prof_${TAG}_writer.log 2>&1 && echo WRITER_OK
}
step_ceil() {
  # the read + record-write ceiling microbenchmark (built on the CPU beforehand), its ONLY_C forms
  ONLY_C=1 timeout -k 10 180 tools/ubench_ceiling > gpurun_out/ceil_${TAG}.txt 2>&1 && cat gpurun_out/ceil_${TAG}.txt
}
step_quick() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTS_K}" \
    > gpurun_out/pytest_${TAG}.log 2>&1 && echo QUICK_OK && tail -3 gpurun_out/pytest_${TAG}.log
}
step_lines() {
  timeout -k 10 180 tools/ubench_lines > gpurun_out/lines_${TAG}.txt 2>&1 && cat gpurun_out/lines_${TAG}.txt
}
step_ab() {
  for c in ${AB_CONFIGS:-get256}; do
    timeout -k 10 ${AB_TIMEOUT:-300} python3 -u tools/ab_libs.py --config $c --rounds ${AB_ROUNDS:-7} --steps ${AB_STEPS:-30} \
      ${AB_ARGS} ${AB_LIBS} > gpurun_out/ab_${TAG}_$c.txt 2>&1 || { tail -5 gpurun_out/ab_${TAG}_$c.txt; return 1; }
    grep "^ab $c\|parity" gpurun_out/ab_${TAG}_$c.txt
  done
}
step_stamps() {
  RHP_LIB=$PWD/libreactorng_amd/librhp_x_stamps.so timeout -k 10 300 python3 tools/stamps2.py > gpurun_out/stamps_${TAG}.txt 2>&1 \
    && grep -v Warning gpurun_out/stamps_${TAG}.txt | head -40
}
step_reactor() {
  timeout -k 10 400 bash tools/reactor_timeline.sh > gpurun_out/reactor_timeline_${TAG}.txt 2>&1 \
    && timeout -k 10 400 python3 tools/reactor_crossover.py > gpurun_out/reactor_crossover_${TAG}_1.txt 2>&1 \
    && timeout -k 10 400 python3 tools/reactor_crossover.py > gpurun_out/reactor_crossover_${TAG}_2.txt 2>&1 \
    && cat gpurun_out/reactor_crossover_${TAG}_1.txt gpurun_out/reactor_crossover_${TAG}_2.txt
}
step_smoke() {
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke_${TAG}.log 2>&1 \
    && tail -1 gpurun_out/smoke_${TAG}.log
}
( ! has quick || step_quick ) && ( ! has lines || step_lines ) && ( ! has ab || step_ab ) && ( ! has stamps || step_stamps ) \
  && ( ! has reactor || step_reactor ) \
  && ( ! has tests || step_tests ) && ( ! has bench || step_bench ) && ( ! has prof || step_prof ) && ( ! has pmc || step_pmc ) \
  && ( ! has sq || step_sq ) && ( ! has writer || step_writer ) && ( ! has smoke || step_smoke ) \
  && ( ! has ceil || step_ceil ) && echo SESSION_OK
