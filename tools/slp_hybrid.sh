#!/bin/bash
# Bisect a flag-dependent miscompare by source file: compile every csrc file of git revision <rev>
# twice (default flags / the variant flags), then link one library per file group with only that
# group built with the variant flags.
# usage: VARIANT_FLAGS=-fno-slp-vectorize tools/slp_hybrid.sh <rev | source dir> <tag> "<group name>:<file> <file>" ...
#   -> fastfourierconvolution_amd/libffc_amd_<tag>_<group>.so, plus <tag>_all (every file) and <tag>_none
set -eu
rev=$1; tag=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
if [ -d "$rev" ]; then   # a source tree (fastfourierconvolution_amd/csrc + include) instead of a revision
  mkdir -p "$tmp/fastfourierconvolution_amd" && cp -r "$rev/fastfourierconvolution_amd/csrc" "$tmp/fastfourierconvolution_amd/" && cp -r "$rev/include" "$tmp/"
else
  git -C "$root" archive "$rev" fastfourierconvolution_amd/csrc include | tar -x -C "$tmp"
fi
src="$tmp/fastfourierconvolution_amd/csrc"
mkdir -p "$tmp/a" "$tmp/b"
pids=()
for f in "$src"/*.hip "$src"/*.cpp; do
  b=$(basename "$f"); x=""; [[ $f == *.cpp ]] && x="-x hip"
  hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $x -c "$f" -o "$tmp/a/$b.o" 2>/dev/null & pids+=($!)
  hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 ${VARIANT_FLAGS:-} $x -c "$f" -o "$tmp/b/$b.o" 2>/dev/null & pids+=($!)
  if [ ${#pids[@]} -ge 8 ]; then wait "${pids[@]}"; pids=(); fi
done
wait
link() {   # link <name> <files built with the variant flags...>
  local name=$1; shift; local objs=()
  for o in "$tmp"/a/*.o; do
    b=$(basename "$o" .o); use=a
    for g in "$@"; do [ "$g" = "$b" ] && use=b; done
    objs+=("$tmp/$use/$b.o")
  done
  hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$root/fastfourierconvolution_amd/libffc_amd_${tag}_$name.so"
  echo "built libffc_amd_${tag}_$name.so ($*)"
}
link none
link all $(cd "$tmp/a" && ls *.o | sed 's/\.o$//')
for spec in "$@"; do link "${spec%%:*}" ${spec#*:}; done
rm -rf "$tmp"
