#!/bin/bash
# Diagnostic library with s_memtime / s_memrealtime stamps in the v9 GEMM (-DSV_CLOCK_STAMPS):
# spine-vision_amd/libsv_kernels_stamp.so, used only by tools/clock_stamp.py through SV_LIB_PATH.
set -eu
cd "$(dirname "$0")/.."
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' -DSV_CLOCK_STAMPS -fno-slp-vectorize \
  -I include -c spine-vision_amd/csrc/gemm9.hip -o $OBJ/gemm9_stamp.o
OBJS=$(ls $OBJ/*.o | grep -v gemm9 )
hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_stamp.so $OBJS $OBJ/gemm9_stamp.o
echo built spine-vision_amd/libsv_kernels_stamp.so
