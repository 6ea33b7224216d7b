#!/bin/bash
# round 5: fused MLP diagnostics, 4-wave workgroups: 1 no GELU, 6 no DMA + no barriers, 14 + weights from registers,
# 15 + no GELU (pure MFMA + the tile's memory traffic)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10h}
mkdir -p $O
for d in 0 1 6 14 15; do
  L=$([ $d = 0 ] && echo spine-vision_amd/libsv_kernels.so || echo spine-vision_amd/libsv_kernels_mlpd$d.so)
  echo "== diag $d" >> $O/mlp_diag.txt
  SV_LIB_PATH=$PWD/$L timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1 >> $O/mlp_diag.txt 2>&1 || { tail -20 $O/mlp_diag.txt; exit 1; }
done
grep -E "==|fused" $O/mlp_diag.txt
