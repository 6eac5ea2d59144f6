#!/bin/bash
# Build libffc_amd_<name>.so from the csrc tree with <file> taken from git revision <rev>.
# usage: [VARIANT_FLAGS="-DX"] tools/build_variant.sh <name> <rev> <csrc file>...   (rev "-" = working tree)
set -eu
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
cp -r "$root/fastfourierconvolution_amd/csrc" "$tmp/csrc"
mkdir -p "$tmp/include" && cp "$root/include/ffc_amd.h" "$tmp/include/"
if [ "$rev" != "-" ]; then
  for f in "$@"; do git -C "$root" show "$rev:fastfourierconvolution_amd/csrc/$f" > "$tmp/csrc/$f"; done
fi
mkdir -p "$tmp/fastfourierconvolution_amd" && mv "$tmp/csrc" "$tmp/fastfourierconvolution_amd/csrc"
objs=()
for src in "$tmp"/fastfourierconvolution_amd/csrc/*.hip "$tmp"/fastfourierconvolution_amd/csrc/*.cpp; do
  o="$tmp/$(basename "$src").o"
  if [[ $src == *.cpp ]]; then x="-x hip"; else x=""; fi
  hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 ${VARIANT_FLAGS:-} $x -c "$src" -o "$o" &
  objs+=("$o")
done
wait
hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$root/fastfourierconvolution_amd/libffc_amd_$name.so"
rm -rf "$tmp"
echo "built libffc_amd_$name.so"
