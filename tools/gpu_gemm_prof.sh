#!/bin/bash
# GEMM microbench + PMC counter passes (one counter group per pass, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-gp}
mkdir -p "$OUT"
ROOTDIR=$(pwd)
timeout -k 10 300 python tools/gemm_bench.py --stages ${STAGES_ARG:-S1,S2,S3,S4} > "$OUT/gemm_bench.txt" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$ROOTDIR/$OUT/counters.txt" 2>&1 || true
i=0
for ctrs in "${PMC_SETS[@]:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$ROOTDIR/$OUT/pmc$i" -o run -- python3 "$ROOTDIR/tools/gemm_bench.py" --stages S3 --iters 3 > "$ROOTDIR/$OUT/pmc$i.log" 2>&1 || exit $?
done
