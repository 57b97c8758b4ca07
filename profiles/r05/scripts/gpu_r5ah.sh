#!/bin/bash
# round 5 session ah: the new large uneven-range test (two order waves) and the line-window tests
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5ah && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_line_windows.py > gpurun_out/r5ah/pytest.log 2>&1 && tail -3 gpurun_out/r5ah/pytest.log && echo SESSION_OK
