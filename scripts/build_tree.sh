#!/bin/bash
# Build libredcliff_hip.so from the working tree's csrc/ + include/ with extra hipcc flags into
# scripts/bin/lib_<name>.so (variant A/B without committing; select with REDCLIFF_HIP_LIB).
#   scripts/build_tree.sh <name> [extra hipcc flags...]
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/redcliff-s-hypothesizing-dynamic-causal-graphs_amd
tmp=$(mktemp -d)
mkdir -p "$root/scripts/bin"
objs=()
for s in "$pkg"/csrc/*.hip; do
  o="$tmp/$(basename "$s").o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$root/include" -I"$pkg/csrc" "$@" -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic "${objs[@]}" -o "$root/scripts/bin/lib_$name.so"
rm -rf "$tmp"
