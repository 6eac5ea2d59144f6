#!/bin/bash
# Build libffc_amd_<name>.so from the working tree with ONE source recompiled under extra flags
# (the other objects from fastfourierconvolution_amd/build_obj).  usage:
#   tools/build_obj_variant.sh <name> <csrc file> <flags...>
set -eu
name=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/fastfourierconvolution_amd
tmp=$(mktemp -d)
hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 "$@" -c "$pkg/csrc/$src" -o "$tmp/$src.o"
objs=()
for o in "$pkg"/build_obj/*.o; do
  [ "$(basename "$o")" = "$src.o" ] && objs+=("$tmp/$src.o") || objs+=("$o")
done
hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$pkg/libffc_amd_$name.so"
rm -rf "$tmp"
echo "built libffc_amd_$name.so ($src $*)"
