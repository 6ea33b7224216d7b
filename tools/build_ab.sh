#!/bin/bash
# A/B library: one source file rebuilt with extra defines, linked with the other objects of the in-tree build,
#   tools/build_ab.sh <tag> <source basename> "<defines>"   ->  spine-vision_amd/libsv_kernels_<tag>.so
# e.g. tools/build_ab.sh auxb gemm9.hip "-DSV_G9_AUXB=1"; use it through SV_LIB_PATH (tools/*_bench.py, bench.py).
set -eu
cd "$(dirname "$0")/.."
TAG=$1; SRC=$2; DEFS=$3
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' $DEFS -fno-slp-vectorize \
  -I include -c spine-vision_amd/csrc/$SRC -o $OBJ/ab_$TAG.o
OBJS=$(ls $OBJ/*.hip.o $OBJ/*.cpp.o | grep -v "/$SRC.o")
hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_$TAG.so $OBJS $OBJ/ab_$TAG.o
echo built spine-vision_amd/libsv_kernels_$TAG.so
