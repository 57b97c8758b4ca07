#!/bin/bash
# round 5 session i: wave-per-session fixup; sessions/reactor parity; reactor timeline and crossover
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5i && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sessions.py tests/test_reactor.py > gpurun_out/r5i/pytest.log 2>&1 && tail -2 gpurun_out/r5i/pytest.log \
 && timeout -k 10 600 bash tools/reactor_timeline.sh > gpurun_out/r5i/reactor_timeline.txt 2>&1 && grep -E "===|H2D|submit|rhp_|D2H|span|awake|per round" gpurun_out/r5i/reactor_timeline.txt \
 && timeout -k 10 900 python tools/reactor_crossover.py --reps 7 > gpurun_out/r5i/reactor_crossover.txt 2>&1 && cat gpurun_out/r5i/reactor_crossover.txt
