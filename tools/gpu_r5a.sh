set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5a && export TMPDIR=/tmp
RHP_LIB=$PWD/libreactorng_amd/librhp_x_stamps.so STAMPS_CFG=2,3,5 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5a/stamps_committed.txt 2>&1 && echo STAMPS_OK \
 && RHP_LIB=$PWD/libreactorng_amd/librhp_x_s260.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest_s260.log 2>&1 && echo PARITY_S260_OK \
 && TAG=r5a LIBS="base s260" ROUNDS=2 bash tools/gpu_ab2.sh > /dev/null 2>&1 && cp gpurun_out/ab_r5a.txt gpurun_out/r5a/ && cat gpurun_out/ab_r5a.txt \
 && for c in get256 zipf post chunked; do TAG=r5a/sq_$c CONFIG=$c bash tools/pmc_sq.sh > gpurun_out/r5a/sq_$c.txt 2>&1 || exit 1; done && echo SQ_OK \
 && TAG=r5a/sq260_get256 CONFIG=get256 RHP_LIB=$PWD/libreactorng_amd/librhp_x_s260.so bash tools/pmc_sq.sh > gpurun_out/r5a/sq260_get256.txt 2>&1 && echo SQ260_OK
