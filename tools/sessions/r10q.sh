#!/bin/bash
# round 5: hand-pipelined LDS fragment reads in the C = 128 fused MLP (SV_MLP_PIPE A/B) -- tests and standalone timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_mlp_fused_gpu.py ${MLPK:+-k "$MLPK"} > $O/t_mlp.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t_mlp.log | head -20; tail -30 $O/t_mlp.log; exit 1; }
grep -cE "PASSED" $O/t_mlp.log
for L in "" $PWD/spine-vision_amd/libsv_kernels_mlpp0.so; do
  echo "== lib ${L:-default}"
  SV_LIB_PATH=$L timeout -k 10 200 python tools/mlp_bench.py --shapes ${SHAPES:-base-S1} --bwd || exit 1
done
