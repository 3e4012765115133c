#!/bin/bash
# Build engine variants for A/B timing (tools/ablate_gpu.sh). Usage: tools/ablate.sh "NAME:-DFLAG -DFLAG2" ...
# NEB_ABLATE_* variants compute WRONG results by design (timing/counter study only).
set -e
cd "$(dirname "$0")/../nebula_amd"
mkdir -p ../build_abl && rm -f ../build_abl/lib_*.so
[ $# -eq 0 ] && set -- "BASE:" "HORNER:-DNEB_ABLATE_HORNER" "FINAL:-DNEB_ABLATE_FINAL" "AES:-DNEB_ABLATE_AES"
: > ../build_abl/variants.txt
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -Wno-unused-result -Wno-unused-value $defs \
     -shared -x hip csrc/aes_gcm.hip -x hip csrc/chacha_poly.hip -x hip csrc/sched.hip -x hip csrc/tx.hip -x hip csrc/rxwin.hip -x hip csrc/engine.cpp -x hip csrc/window.cpp -o ../build_abl/lib_$name.so &
  echo $name >> ../build_abl/variants.txt
done
wait
ls ../build_abl
