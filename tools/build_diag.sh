#!/bin/bash
# Diagnostic library: the v9 GEMM with its epilogue's memory instructions compiled out (-DSV_DIAG_NOSTORE),
# spine-vision_amd/libsv_kernels_nostore.so -- tools/gemm_bench.py through SV_LIB_PATH times the K loop alone.
set -eu
cd "$(dirname "$0")/.."
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' -DSV_DIAG_NOSTORE -fno-slp-vectorize \
  -I include -c spine-vision_amd/csrc/gemm9.hip -o $OBJ/gemm9_nostore.o
OBJS=$(ls $OBJ/*.o | grep -v gemm9 )
hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_nostore.so $OBJS $OBJ/gemm9_nostore.o
echo built spine-vision_amd/libsv_kernels_nostore.so
