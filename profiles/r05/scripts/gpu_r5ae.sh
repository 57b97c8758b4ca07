#!/bin/bash
# round 5 session ae: chunked -- the group build not unrolled over the four bodies (nu: less code in the moves loop)
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5ae && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
RHP_LIB=$L/librhp_x_nu.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "chunk or golden" > gpurun_out/r5ae/pytest_nu.log 2>&1 && tail -1 gpurun_out/r5ae/pytest_nu.log || exit 1
for r in 1 2 3; do
  for v in cur nu; do
    for c in chunked post; do
      RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5ae/${c}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r5ae/${c}_$v.json')); print('$v', '$c', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5ae/ab.txt
    done
  done
done
echo SESSION_OK
