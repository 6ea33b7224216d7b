#!/bin/bash
# Diagnostic libraries for the fused MLP (csrc/mlp.hip, -DSV_MLP_DIAG=1/2/3): spine-vision_amd/libsv_kernels_mlpdN.so,
# loaded through SV_LIB_PATH by tools/mlp_bench.py (timing only: their results are wrong)
set -eu
cd "$(dirname "$0")/.."
OBJ=spine-vision_amd/build
python -c "import __graft_entry__ as g; g.build_native()"
for d in ${DIAGS:-1 2 3}; do
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DSV_OFFLOAD_ARCH='"gfx950"' -DSV_MLP_DIAG=$d -fno-slp-vectorize \
    -I include -c spine-vision_amd/csrc/mlp.hip -o $OBJ/mlp_d$d.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o spine-vision_amd/libsv_kernels_mlpd$d.so $(ls $OBJ/*.hip.o $OBJ/*.cpp.o | grep -v "mlp.hip.o") \
    $OBJ/mlp_d$d.o
done
echo built
