#!/bin/bash
# Build a measurement variant of libdrhip.so: one csrc/<unit>.hip recompiled
# with extra -D flags, the other objects reused from distributed-ranges_amd/build.
# usage: tools/build_variant.sh <name> <unit> "<flags>"  ->  tools/var/<name>/libdrhip.so
set -e
cd "$(dirname "$0")/../distributed-ranges_amd"
name=$1 unit=$2 flags=$3
out=../tools/${VAR_ROOT:-var}/$name
rm -rf "$out" && mkdir -p "$out/build"
for f in csrc/*.hip; do
  b=$(basename "$f" .hip)
  if [ "$b" = "$unit" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off $flags \
      -c "$f" -o "$out/build/$b.o"
  else
    cp "build/$b.o" "$out/build/"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libdrhip.so" "$out"/build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$out/build"
echo "$out/libdrhip.so"
