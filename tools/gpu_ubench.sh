set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 ./tools/ubench_stream > gpurun_out/ubench_stream.txt 2>&1 && cat gpurun_out/ubench_stream.txt \
 && timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ub_fetch -o p -- ./tools/ubench_stream pmc > gpurun_out/ub_fetch.log 2>&1 \
 && echo UB_PMC_OK \
 && RHP_BENCH_DIAG=1 timeout -k 10 300 python bench.py --extra none --no-cpu --no-e2e > gpurun_out/bench_diag.json 2> gpurun_out/bench_diag.err \
 && cat gpurun_out/bench_diag.json && grep "bench diag" gpurun_out/bench_diag.err
