#!/bin/bash
# round 5 session g: reactor round timeline after the warm-up copies; crossover
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5g && export TMPDIR=/tmp
timeout -k 10 600 bash tools/reactor_timeline.sh > gpurun_out/r5g/reactor_timeline.txt 2>&1 && grep -E "===|H2D|submit|rhp_|D2H|span|awake|per round" gpurun_out/r5g/reactor_timeline.txt \
 && timeout -k 10 900 python tools/reactor_crossover.py --reps 7 > gpurun_out/r5g/reactor_crossover.txt 2>&1 && cat gpurun_out/r5g/reactor_crossover.txt
