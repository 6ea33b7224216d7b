#!/bin/bash
# standalone GEMM shapes of the ConvNeXt-base step (tools/gemm_bench.py), all stages
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gstd}
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/gemm_bench.py --stages ${STAGES:-S1,S2,S3,S4} --iters 20 ${GB_ARGS:-} > "$OUT/gemm.txt" 2> "$OUT/gemm.err"
rc=$?; echo "gemm rc=$rc"; cat "$OUT/gemm.txt"
exit $rc
