#!/bin/bash
# Diagnostic variant with every object rebuilt (header-level macros): tools/build_variant_full.sh NAME "-DX=..."
# -> openwhisk_amd/variants/libowgs_NAME.so (OWGS_LIB=...; never used by tests, smoke or bench)
set -e
cd "$(dirname "$0")/../openwhisk_amd"
mkdir -p variants build/variants/$1
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $2"
for f in owgs_kernels owgs_engine_narrow owgs_watch owgs_fused owgs_resident owgs_seq owgs_state owgs_acks owgs_health owgs_msgs; do
  /opt/rocm/bin/hipcc $F -c -o build/variants/$1/$f.o csrc/$f.hip &
done
/opt/rocm/bin/hipcc $F -x hip -c -o build/variants/$1/owgs_host.o csrc/owgs_host.cpp
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libowgs_$1.so build/variants/$1/*.o
