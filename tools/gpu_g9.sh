#!/bin/bash
# v9 GEMM: family parity test, then standalone timings (impl 0 = dispatch vs 9)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-g9}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_family_gpu.py > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 400 python -u tools/gemm_bench.py --stages ${STAGES:-S1,S2,S3,S4} --iters 20 --impls 0,9 --cases ${CASES:-fc} > "$OUT/gemm.txt" 2> "$OUT/gemm.err"
rc=$?; echo "gemm rc=$rc"; cat "$OUT/gemm.txt"; tail -3 "$OUT/gemm.err"
exit $rc
