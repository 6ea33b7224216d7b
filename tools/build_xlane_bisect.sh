#!/bin/bash
# Bisection builds of the fused MLP backward's cross-lane epilogue (csrc/mlp.hip SV_MLPB_XLANE bits):
# spine-vision_amd/libsv_kernels_xlN.so, loaded through SV_LIB_PATH by tools/mlp_bwd_diag.py
set -eu
cd "$(dirname "$0")/.."
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
for d in ${XL:-1 2 3}; do
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' -DSV_MLPB_XLANE=$d \
    -I include -c spine-vision_amd/csrc/mlp.hip -o $OBJ/mlp_xl$d.o &
done
wait
for d in ${XL:-1 2 3}; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_xl$d.so \
    $(ls $OBJ/*.hip.o $OBJ/*.cpp.o | grep -v "/mlp.hip.o") $OBJ/mlp_xl$d.o
done
echo built
