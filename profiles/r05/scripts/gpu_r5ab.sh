#!/bin/bash
# round 5 session ab: a second reactor crossover run on the committed tree
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5ab && export TMPDIR=/tmp
timeout -k 10 900 python tools/reactor_crossover.py --reps 7 > gpurun_out/r5ab/reactor_crossover.txt 2>&1 && cat gpurun_out/r5ab/reactor_crossover.txt && echo SESSION_OK
