#!/bin/bash
# round 5 session j: line-aligned first windows (S_PRE) -- GPU parity, then A/B against the previous kernel
# (configs 2/3/5) and FETCH_SIZE / WRITE_SIZE of config 3 for both
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5j && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r5j/pytest_parity.log 2>&1 && tail -2 gpurun_out/r5j/pytest_parity.log || exit 1
for v in base line base line; do
  for c in get256 zipf post; do
    RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5j/${c}_$v.json 2>/dev/null || exit 1
  done
  python3 -c "
import json
r=[json.load(open(f'gpurun_out/r5j/{c}_$v.json')) for c in ('get256','zipf','post')]
print('$v', ' '.join(f\"{c} {d['roofline']['kernel_ms']*1e3:.1f}us\" for c,d in zip(('c2','c3','c5'),r)), [list(d['parity'].values()) for d in r])" | tee -a gpurun_out/r5j/ab.txt
done
for v in base line; do
  for k in FETCH_SIZE WRITE_SIZE; do
    RHP_LIB=$L/librhp_x_$v.so timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d gpurun_out/r5j/pmc_${v}_zipf_$k -o p \
      -- python3 bench.py --config zipf --extra none --steps 6 --warmup 2 --no-cpu --no-e2e > gpurun_out/r5j/pmc_${v}_zipf_$k.log 2>&1 || exit 1
  done
done
echo SESSION_OK
