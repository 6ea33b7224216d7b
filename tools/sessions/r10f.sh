#!/bin/bash
# round 5: fused MLP diagnostic builds (no GELU / no weight DMA / neither) against the real one, standalone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10f}
mkdir -p $O
for d in 0 1 2 3; do
  L=$([ $d = 0 ] && echo spine-vision_amd/libsv_kernels.so || echo spine-vision_amd/libsv_kernels_mlpd$d.so)
  echo "== diag $d" | tee -a $O/mlp_diag.txt
  SV_LIB_PATH=$PWD/$L timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1,base-S2 >> $O/mlp_diag.txt 2>&1 || { tail -20 $O/mlp_diag.txt; exit 1; }
done
grep -E "==|fused" $O/mlp_diag.txt
