#!/bin/bash
# shader clock + launch time of the DFA kernel and its timing-experiment builds
set -o pipefail
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
out=gpurun_out/kclock.txt; : > $out
for lib in clock clk_nodec clk_nostep clk_mem; do
  echo "== librhp_$lib" >> $out
  RHP_LIB=$PWD/libreactorng_amd/librhp_$lib.so timeout -k 10 200 python tools/kclock.py >> $out 2>&1 || exit 1
done
for w in 8 12; do
  echo "== librhp_clock RHP_WAVES=$w" >> $out
  RHP_WAVES=$w RHP_LIB=$PWD/libreactorng_amd/librhp_clock.so timeout -k 10 200 python tools/kclock.py >> $out 2>&1 || exit 1
done
grep -v amdgpu.ids $out
