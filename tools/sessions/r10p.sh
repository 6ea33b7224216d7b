#!/bin/bash
# round 5: C = 512 fused MLP diagnostic builds (tools/build_mlp_diag.sh): what bounds the S3 kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10p}
mkdir -p $O
for d in 0 ${DIAGS:-1 2 4 8 15}; do
  L=""; [ $d != 0 ] && L=$PWD/spine-vision_amd/libsv_kernels_mlpd$d.so
  echo "== diag $d"
  SV_LIB_PATH=$L timeout -k 10 120 python tools/mlp_bench.py --shapes base-S3 || exit 1
done
