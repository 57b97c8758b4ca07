#!/bin/bash
# round 5 session q: chunked -- the group's blocks built flattened across its bodies (5 trips per group, chunk by
# compare count + one LDS record) against body by body; parity first
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/r5q && export TMPDIR=/tmp
L=$PWD/libreactorng_amd
RHP_LIB=$L/librhp_x_flat.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_staged_moves_model.py tests/test_line_windows.py > gpurun_out/r5q/pytest_flat.log 2>&1 && tail -2 gpurun_out/r5q/pytest_flat.log || exit 1
for r in 1 2; do
  for v in cur flat; do
    for c in chunked post; do
      RHP_LIB=$L/librhp_x_$v.so timeout -k 10 300 python bench.py --config $c --extra none --no-cpu --no-e2e --steps 30 --warmup 5 > gpurun_out/r5q/${c}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r5q/${c}_$v.json')); print('$v', '$c', round(d['roofline']['kernel_ms']*1e3,1), 'us', d['parity'])" | tee -a gpurun_out/r5q/ab.txt
    done
  done
done
echo SESSION_OK
