#!/bin/bash
# v10 (128x256, two staggered workgroups per CU): bitwise family tests, then timing against v9 (impl 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4f}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_family_gpu.py > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
CASES="fc1_fwd(dual),fc1_fwd(store),fc2_fwd(res),fc2_dgrad(mul),fc1_dgrad,fc2_wgrad+bias,fc1_wgrad"
timeout -k 10 400 python tools/gemm_bench.py --stages S1,S2,S3,S4 --iters 10 --impls 0,10 --cases "$CASES" > "$OUT/gemm.txt" 2>&1
rc=$?; echo "gemm rc=$rc"; grep -v amdgpu.ids "$OUT/gemm.txt"
for st in 0 2 8; do
  SV_G10_STAGGER=$st timeout -k 10 200 python tools/gemm_bench.py --stages S3 --iters 10 --impls 10 --cases "fc1_fwd(dual),fc2_dgrad(mul),fc1_dgrad" > "$OUT/gemm_st$st.txt" 2>&1
  echo "stagger $st"; grep -v amdgpu.ids "$OUT/gemm_st$st.txt"
done
exit 0
