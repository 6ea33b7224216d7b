#!/bin/bash
# fp32 conv diagnostic + PMC passes over the S3 GEMM classes (standalone)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r2f}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/diag_rn_fp32.py > "$OUT/diag.log" 2>&1
rc=$?; echo "diag rc=$rc"; [ $rc -gt 1 ] && exit $rc
GB_ARGS="--stages S3 --iters 3 --cases fc1_fwd(dual),fc2_fwd(res),fc2_dgrad(mul),fc1_dgrad,fc2_wgrad+bias,fc1_wgrad" bash tools/gemm_pmc.sh "$(basename $OUT)/pmc"
