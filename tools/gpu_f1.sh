set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG:-f1}.log 2>&1 && echo PYTEST_OK || { tail -40 gpurun_out/pytest_${TAG:-f1}.log; exit 1; }
TAG=${TAG:-ab6} REPS=3 LIBS="librhp_base librhp" CFGS="${CFGS:-post get256 zipf}" bash tools/ab.sh
