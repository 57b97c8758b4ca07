#!/bin/bash
# round 5 session e: the reactor round's blocking H2D call, by completion mode
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5e && export TMPDIR=/tmp
for mode in event spin hostfunc; do
  echo "=== RHP_REACTOR_COMPLETE=$mode"
  RHP_REACTOR_COMPLETE=$mode RHP_REACTOR_PARSER=gpu RHP_REACTOR_STATS=2 timeout -k 10 120 libreactorng_amd/bin/burst_test 64 64 7 2>&1 \
    | grep -E "H2D|submit|launches|device span|awake|per round" || exit 1
done
