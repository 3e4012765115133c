#!/bin/bash
# Build ablation variants of the engine (results WRONG by design; timing/counter study only).
set -e
cd "$(dirname "$0")/../nebula_amd"
mkdir -p ../build_abl
for v in BASE HORNER FINAL AES; do
  def=""; [ "$v" != BASE ] && def="-DNEB_ABLATE_$v"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wno-unused-result $def \
     -shared -x hip csrc/aes_gcm.hip -x hip csrc/chacha_poly.hip -x hip csrc/sched.hip -x hip csrc/engine.cpp -o ../build_abl/lib_$v.so
done
ls -la ../build_abl
