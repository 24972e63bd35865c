#!/bin/bash
# Build a libppox variant with extra -D flags for kernel A/B timing (dev tool).
# Usage: tools/build_variant.sh NAME "-DFC_NB=128 -DWS_KT2=64"
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/variants/$name
mkdir -p "$out"
objs=()
for f in "$root"/ppo-exploration_amd/csrc/*.hip "$root"/ppo-exploration_amd/csrc/*.cpp; do
  o=$out/$(basename "$f").o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics \
    -I"$root/include" $* -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libppox.so" "${objs[@]}"
echo "$out/libppox.so"
