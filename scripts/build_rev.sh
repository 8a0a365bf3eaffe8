#!/bin/bash
# Build libredcliff_hip.so from the csrc/ + include/ of a git revision into scripts/bin/lib_<name>.so
# (A/B and bitwise comparisons against an earlier build; select with REDCLIFF_HIP_LIB).
#   scripts/build_rev.sh <rev> <name> [extra hipcc flags...]
set -e
rev=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
pkg=redcliff-s-hypothesizing-dynamic-causal-graphs_amd
mkdir -p "$tmp/csrc" "$tmp/include" "$root/scripts/bin"
for f in $(git -C "$root" ls-tree --name-only "$rev" $pkg/csrc/ include/); do
  git -C "$root" show "$rev:$f" > "$tmp/${f#$pkg/}"
done
objs=()
for s in "$tmp"/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$tmp/include" -I"$tmp/csrc" "$@" -c "$s" -o "$s.o" &
  objs+=("$s.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic "${objs[@]}" -o "$root/scripts/bin/lib_$name.so"
rm -rf "$tmp"
echo "$root/scripts/bin/lib_$name.so"
