#!/bin/bash
# round 5 session k: config 3 after line windows -- waves, cache policy, record layouts; stamps of configs 2/3;
# config 5 (compact http records) WRITE_SIZE / FETCH_SIZE
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5k && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
run() {  # name lib layout
  RHP_LIB=$L/librhp_x_$2.so RHP_BENCH_LAYOUTS="zipf=$3" timeout -k 10 300 python bench.py --config zipf --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5k/$1.json 2>/dev/null || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/r5k/$1.json')); print('$1', round(d['roofline']['kernel_ms']*1e3,1), 'us', round(d['ms_per_step']*1e3,1), d['parity'])" | tee -a gpurun_out/r5k/ab.txt
}
for r in 1 2; do
  run line_req line request && run nont nont request \
   && run line_hdr line header && run line_cmp line compact || exit 1
done
RHP_LIB=$L/librhp_x_stamps.so STAMPS_CFG=2,3 timeout -k 10 240 python tools/stamps2.py > gpurun_out/r5k/stamps.txt 2>&1 && echo STAMPS_OK || exit 1
for k in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d gpurun_out/r5k/pmc_post_$k -o p \
    -- python3 bench.py --config post --extra none --steps 6 --warmup 2 --no-cpu --no-e2e > gpurun_out/r5k/pmc_post_$k.log 2>&1 || exit 1
done
echo SESSION_OK
