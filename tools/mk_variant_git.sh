#!/bin/bash
# Build a variant library from the working tree with some files taken from a git revision:
# tools/mk_variant_git.sh <name> <rev> <path>... [-- extra compile flags]
set -e
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
dst=$root/tools/_var_$name
rm -rf "$dst" && mkdir -p "$dst"
cp -r "$root/suffix-array-searching_amd" "$dst/"
cp -r "$root/include" "$dst/"
rm -rf "$dst/suffix-array-searching_amd/build" "$dst/suffix-array-searching_amd/libsas_amd.so"
flags=""
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; flags="$*"; break; fi
  git -C "$root" show "$rev:$1" > "$dst/$1"
  shift
done
make -s -j8 -C "$dst/suffix-array-searching_amd" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $flags"
rm -rf "$dst/suffix-array-searching_amd/build"
