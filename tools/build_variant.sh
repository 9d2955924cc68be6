#!/bin/bash
# Diagnostic engine variants: tools/build_variant.sh NAME "-DKPROBE=8 ..." -> openwhisk_amd/variants/libowgs_NAME.so
# (select one at run time with OWGS_LIB=...; never used by tests, smoke or bench).  Only the main engine object and
# the host are rebuilt with the flags; the other objects come from the regular build.
set -e
cd "$(dirname "$0")/../openwhisk_amd"
mkdir -p variants build/variants
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2"
/opt/rocm/bin/hipcc $F -c -o build/variants/k_$1.o csrc/owgs_kernels.hip
/opt/rocm/bin/hipcc $F -x hip -c -o build/variants/h_$1.o csrc/owgs_host.cpp
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libowgs_$1.so build/variants/k_$1.o \
  build/owgs_engine_narrow.o build/owgs_watch.o build/owgs_fused.o build/owgs_state.o build/owgs_acks.o \
  build/owgs_health.o build/owgs_msgs.o build/variants/h_$1.o
