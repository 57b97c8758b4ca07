#!/bin/bash
# Build librhp.so as it was at a git commit, for same-box A/B runs:
#   tools/build_at.sh <commit> <tag>  ->  libreactorng_amd/librhp_x_<tag>.so
# (bench.py / tools take it through RHP_LIB=...; the batch ABI of include/rhp.h
# is the same since round 4)
set -e
c=$1; tag=$2
root=$(git rev-parse --show-toplevel)
d=$(mktemp -d /tmp/build_at.XXXXXX)
git -C "$root" archive "$c" include libreactorng_amd/csrc | tar -x -C "$d"
make -s -C "$d/libreactorng_amd/csrc" ../librhp.so
cp "$d/libreactorng_amd/librhp.so" "$root/libreactorng_amd/librhp_x_$tag.so"
rm -rf "$d"
echo "built libreactorng_amd/librhp_x_$tag.so from $c"
