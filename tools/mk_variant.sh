#!/bin/bash
# Build a variant of libsas_amd.so with extra compile flags into tools/_var_<name>/
# (package copy + library), for same-box A/B runs: tools/mk_variant.sh nt2 -DSAS_QUAD_NT_LEVELS=2
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/tools/_var_$name
rm -rf "$dst" && mkdir -p "$dst"
cp -r "$root/suffix-array-searching_amd" "$dst/"
cp -r "$root/include" "$dst/"
rm -rf "$dst/suffix-array-searching_amd/build" "$dst/suffix-array-searching_amd/libsas_amd.so"
make -s -j8 -C "$dst/suffix-array-searching_amd" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*"
rm -rf "$dst/suffix-array-searching_amd/build"
