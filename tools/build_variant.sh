#!/bin/bash
# Builds variants/NAME/libzsgpu.so: the in-tree objects with ONE source recompiled
# under extra defines (timing / instrumentation experiments):
#   tools/build_variant.sh NAME SOURCE.hip -DMACRO=V ...
set -e
cd "$(dirname "$0")/../zlib-streams-ts_amd/csrc"
name=$1; src=$2; shift 2
make -s -j8 >/dev/null
mkdir -p ../../variants/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function "$@" -x hip -c $src -o ../../variants/$name/$src.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../variants/$name/libzsgpu.so $(ls build/*.o | grep -v "build/$src.o") ../../variants/$name/$src.o
echo variants/$name/libzsgpu.so
