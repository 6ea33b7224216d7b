#!/bin/bash
# A/B libraries of the v9 GEMM's K-loop wave priority (SV_G9_PRIO = 1: static priority for waves 4-7;
# 2: no s_setprio) -> spine-vision_amd/libsv_kernels_prio{1,2}.so, used through SV_LIB_PATH
set -eu
cd "$(dirname "$0")/.."
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
OBJS=$(ls $OBJ/*.o | grep -v gemm9 )
for p in ${PRIOS:-1 2}; do
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' -DSV_G9_PRIO=$p -fno-slp-vectorize \
    -I include -c spine-vision_amd/csrc/gemm9.hip -o $OBJ/gemm9_prio$p.o.tmp
  hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_prio$p.so $OBJS $OBJ/gemm9_prio$p.o.tmp
  rm -f $OBJ/gemm9_prio$p.o.tmp
  echo built spine-vision_amd/libsv_kernels_prio$p.so
done
