#!/bin/bash
# Build an A/B variant of libnebula_aead.so with extra -D flags into build_var/<name>/ (CPU side;
# the .so travels to the GPU box). Use it with NEB_LIB_PATH=build_var/<name>/libnebula_aead.so.
#   tools/build_variant.sh <name> -DFLAG=1 ...
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
out=$R/build_var/$name
mkdir -p "$out"
cd "$R/nebula_amd"
make -s -j8 BUILD="$out/obj" LIB="$out/libnebula_aead.so" HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-value -fvisibility=hidden $*" "$out/libnebula_aead.so"
echo "$out/libnebula_aead.so"
