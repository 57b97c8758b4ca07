#!/bin/bash
# round 5 session l: chunked bodies validated from their LDS slots -- GPU parity, chunked/config 5 A/B, traffic
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5l && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r5l/pytest_parity.log 2>&1 && tail -2 gpurun_out/r5l/pytest_parity.log || exit 1
for v in line slot line slot; do
  for c in chunked post; do
    RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5l/${c}_$v.json 2>/dev/null || exit 1
  done
  python3 -c "
import json
r=[json.load(open(f'gpurun_out/r5l/{c}_$v.json')) for c in ('chunked','post')]
print('$v', ' '.join(f\"{c} {d['roofline']['kernel_ms']*1e3:.1f}us\" for c,d in zip(('chunked','c5'),r)), [list(d['parity'].values()) for d in r])" | tee -a gpurun_out/r5l/ab.txt
done
for k in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d gpurun_out/r5l/pmc_slot_chunked_$k -o p \
    -- python3 bench.py --config chunked --extra none --steps 6 --warmup 2 --no-cpu --no-e2e > gpurun_out/r5l/pmc_slot_chunked_$k.log 2>&1 || exit 1
done
echo SESSION_OK
