#!/bin/bash
# Per-phase timeline of the reactor's GPU rounds: burst_test
# at 4K, 16K and 64K-request rounds with RHP_REACTOR_STATS=2 (batch.c: H2D,
# parse, fix-up, D2H from events on the round's stream; the completion thread's
# wake-up and the loop's pick-up from host clocks; server.c: pack and dispatch;
# core.c: time blocked in epoll_wait), the host parser beside it.
# usage: bash tools/reactor_timeline.sh > gpurun_out/reactor_timeline.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
B=libreactorng_amd/bin/burst_test
for size in "64 64" "128 128" "256 256"; do
  for parser in gpu host; do
    echo "=== round ${size// / x } parser $parser"
    RHP_REACTOR_PARSER=$parser RHP_REACTOR_STATS=2 timeout -k 10 120 $B $size 7 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
