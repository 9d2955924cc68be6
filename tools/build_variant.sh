#!/bin/bash
# Diagnostic engine variants: tools/build_variant.sh NAME "-DKPROBE=8 ..." -> openwhisk_amd/variants/libowgs_NAME.so
# (select one at run time with OWGS_LIB=...; never used by tests, smoke or bench).  The engine objects (wide and
# narrow geometry) and the host are rebuilt with the flags; the other objects come from the regular build.
set -e
cd "$(dirname "$0")/../openwhisk_amd"
mkdir -p variants build/variants
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-unroll-loops $2"  # (as the Makefile builds the engine)
rm -f build/variants/k_$1.o build/variants/n_$1.o build/variants/h_$1.o
/opt/rocm/bin/hipcc $F -c -o build/variants/k_$1.o csrc/owgs_kernels.hip & p1=$!
# (the narrow geometry too: the host must see the same geometry macros as every engine object it launches)
/opt/rocm/bin/hipcc $F -c -o build/variants/n_$1.o csrc/owgs_engine_narrow.hip & p2=$!
/opt/rocm/bin/hipcc $F -x hip -c -o build/variants/h_$1.o csrc/owgs_host.cpp & p3=$!
wait $p1 && wait $p2 && wait $p3
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libowgs_$1.so build/variants/k_$1.o \
  build/variants/n_$1.o build/owgs_watch.o build/owgs_fused.o build/owgs_resident.o build/owgs_seq.o build/owgs_state.o build/owgs_acks.o \
  build/owgs_health.o build/owgs_msgs.o build/variants/h_$1.o
