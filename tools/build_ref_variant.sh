#!/bin/bash
# A/B helper: build the engine of git revision $1 as openwhisk_amd/variants/libowgs_$2.so
set -e
REV=$1; NAME=$2; shift 2
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d)
mkdir -p $T/openwhisk_amd/csrc $T/include
for f in csrc/owgs_kernels.hip csrc/owgs_internal.h csrc/owgs_host.cpp; do git -C "$ROOT" show $REV:openwhisk_amd/$f > $T/openwhisk_amd/$f; done
git -C "$ROOT" show $REV:include/owgs.h > $T/include/owgs.h
mkdir -p "$ROOT/openwhisk_amd/variants"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
cd $T/openwhisk_amd
/opt/rocm/bin/hipcc $F -c -o k.o csrc/owgs_kernels.hip
/opt/rocm/bin/hipcc $F -x hip -c -o h.o csrc/owgs_host.cpp
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/openwhisk_amd/variants/libowgs_$NAME.so" k.o h.o
rm -rf $T
