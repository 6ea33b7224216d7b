#!/bin/bash
# cross-lane fused-MLP-backward bisection, second step: XLANE=3 with vm_wait<0> before the epilogue (d1) and with
# every compiler wait forced to zero (fz)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r15b}
mkdir -p $O
for v in _xl3d1 _xl3fz; do
  SV_LIB_PATH=$PWD/spine-vision_amd/libsv_kernels$v.so timeout -k 10 240 python -u tools/mlp_bwd_diag.py 524288 524288 > $O/diag$v.txt 2>&1 || { tail -20 $O/diag$v.txt; exit 1; }
  echo "== lib$v"; grep "deterministic\|differing" $O/diag$v.txt
done
