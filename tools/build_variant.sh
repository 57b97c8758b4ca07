#!/bin/bash
# Build librhp.so from the working tree with extra compile flags, for same-box
# A/B runs (tools/ab_libs.py):
#   tools/build_variant.sh <tag> -DRHP_DIAG_EXTRA_LDS ...  ->  libreactorng_amd/librhp_x_<tag>.so
set -e
tag=$1; shift
root=$(git rev-parse --show-toplevel)
cd "$root/libreactorng_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fconstexpr-steps=50000000 -DRHP_BLOCK=128 -DRHP_WAVES_PER_SIMD=4 \
  "$@" -I../../include -I. -fPIC -shared rhp_kernel.hip rhp_writer.hip -o "../librhp_x_$tag.so"
echo "built libreactorng_amd/librhp_x_$tag.so ($*)"
