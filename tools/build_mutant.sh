#!/bin/bash
# Mutation variants of libppox for the tests (dev tool): a copy of the sources with ONE deliberate numerical
# fault, built as tools/variants/NAME/libppox.so.  The tests that guard against the fault must FAIL on it
# (tools/gpu.sh step xfail:NAME:FILE[:K]); the product sources are untouched.
#   flushlo1: the conv1 forward's packed weights lose every subnormal low f16 plane (the weights below
#             2^-17 of the tensor's max lose their low 11 bits: csrc/conv_common.h pack_fwd1_split_elem)
# Usage: tools/build_mutant.sh flushlo1
set -e
name=$1
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/pkg" && cp -r "$root/ppo-exploration_amd/csrc" "$tmp/pkg/csrc"  # csrc/common.h: ../../include
mkdir -p "$tmp/include" && cp "$root/include/"*.h "$tmp/include/"
case $name in
  flushlo1)
    f=$tmp/pkg/csrc/conv_common.h
    grep -q 'q\[fwd1_split_index(c, st, 1, lane, e)\] = p1;' "$f"
    sed -i 's/q\[fwd1_split_index(c, st, 1, lane, e)\] = p1;/q[fwd1_split_index(c, st, 1, lane, e)] = (p1 \& 0x7c00) ? p1 : (uint16_t)0;/' "$f"
    grep -q '(p1 & 0x7c00) ? p1' "$f" ;;
  *) echo "unknown mutant $name" >&2; exit 2 ;;
esac
out=$root/tools/variants/$name
mkdir -p "$out"
objs=()
for f in "$tmp"/pkg/csrc/*.hip "$tmp"/pkg/csrc/*.cpp; do
  o=$tmp/$(basename "$f").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics \
    -I"$tmp/include" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libppox.so.tmp" "${objs[@]}"
mv "$out/libppox.so.tmp" "$out/libppox.so"
echo "$out/libppox.so"
