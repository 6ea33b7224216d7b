#!/bin/bash
# round 6: is the cross-lane mlpb128 non-determinism a v_permlane*_swap write -> VALU read hazard?  The same kernel
# built twice: libsv_kernels_xl.so (cross-lane epilogue, as r13b: dz rows differed run to run) and
# libsv_kernels_xl2.so (the same with 5 wait states between every permlane swap and the read of its results,
# -DSV_PERMLANE_NOP=5).  The run-to-run test (4 runs each, names what differs), twice per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
O=$ROOTDIR/gpurun_out/${1:-r13c}
mkdir -p $O
for lib in xl2 xl xl2 xl; do
  SV_LIB_PATH=$ROOTDIR/spine-vision_amd/libsv_kernels_$lib.so timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_mlp_fused_gpu.py -k "bwd_fused_matches and base-S1" > $O/$lib.log 2>&1
  echo "$lib: exit $? $(grep -oE '[0-9]+ (passed|failed)' $O/$lib.log | tr '\n' ' ') $(grep -oE 'd[zhwb] differs[^;]*' $O/$lib.log | head -1)"
done
