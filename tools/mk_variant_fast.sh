#!/bin/bash
# Like mk_variant.sh, but only sas_search.hip is rebuilt with the extra flags; the other
# objects come from the main in-tree build (make it first).
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/tools/_var_$name
rm -rf "$dst" && mkdir -p "$dst"
cp -r "$root/suffix-array-searching_amd" "$dst/"
cp -r "$root/include" "$dst/"
rm -f "$dst/suffix-array-searching_amd/libsas_amd.so" "$dst/suffix-array-searching_amd/build/sas_search.o"
touch "$dst"/suffix-array-searching_amd/build/*.o
make -s -C "$dst/suffix-array-searching_amd" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*"
rm -rf "$dst/suffix-array-searching_amd/build"
