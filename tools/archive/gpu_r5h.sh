#!/bin/bash
# round 3, session 3: the N = 128 GEMMs (S1 fc1 dgrad on v3, S1 fc2 residual on v2) forced onto v9 (half-filled
# 256-wide tiles) against the dispatch, standalone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5h}
mkdir -p "$OUT"
timeout -k 10 300 python tools/gemm_bench.py --cases "fc1_dgrad,fc2_fwd(res),fc1_wgrad,fc2_wgrad" --stages S1 --impls 0,9,3,2 > "$OUT/gemm.txt" 2>&1
rc=$?; echo "gemm rc=$rc"; grep -v amdgpu "$OUT/gemm.txt"
exit $rc
