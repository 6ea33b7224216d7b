#!/bin/bash
# cross-lane fused-MLP-backward bisection, third step: the x-hat operands pinned below the epilogue's counted wait
# (SV_MLPB_PIN, default and XLANE=3), the unpinned XLANE=3 as the control on the same box; the fused-MLP tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r15c}
mkdir -p $O
for v in "" _xl3p _xl3; do
  SV_LIB_PATH=$PWD/spine-vision_amd/libsv_kernels$v.so timeout -k 10 240 python -u tools/mlp_bwd_diag.py 524288 524288 524288 > $O/diag$v.txt 2>&1 || { tail -20 $O/diag$v.txt; exit 1; }
  echo "== lib$v"; grep "deterministic\|differing" $O/diag$v.txt
done
timeout -k 10 600 python -u -m pytest tests/test_mlp_fused_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_mlp.txt 2>&1 || { tail -30 $O/t_mlp.txt; exit 1; }
tail -2 $O/t_mlp.txt
