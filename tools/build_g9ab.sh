#!/bin/bash
# A/B library: the v9 GEMM with the 16-row x 64-B epilogue access shape (-DSV_G9_ROWS128=0),
# spine-vision_amd/libsv_kernels_r64.so -- tools/gemm_bench.py / bench.py through SV_LIB_PATH.
set -eu
cd "$(dirname "$0")/.."
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' -DSV_G9_ROWS128=0 -fno-slp-vectorize \
  -I include -c spine-vision_amd/csrc/gemm9.hip -o $OBJ/gemm9_r64.o
OBJS=$(ls $OBJ/*.o | grep -v gemm9 )
hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_r64.so $OBJS $OBJ/gemm9_r64.o
echo built spine-vision_amd/libsv_kernels_r64.so
