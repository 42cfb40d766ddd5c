#!/bin/bash
# Build librein48 with one source file replaced (experiments): tools/build_variant.sh <variant.hip> <replaced object name> <out.so> [extra hipcc flags]
set -e
V=$1; NAME=$2; OUT=$3; shift 3
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function "$@" -I rein48_amd/csrc -c -o build/var/$NAME.var.o -x hip $V
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -o $OUT $(ls build/obj/*.o | grep -v "/$NAME.o") build/var/$NAME.var.o
