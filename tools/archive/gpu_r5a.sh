#!/bin/bash
# round 3, session 3: full -m gpu suite on the restored tree, standalone depthwise timings, PMC passes
# over the depthwise kernels at S1/S3 (what bounds them: VALU issue vs memory wait)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 300 python tools/dw_bench.py > "$OUT/dw.txt" 2>&1
rc=$?; echo "dw rc=$rc"; grep -v amdgpu "$OUT/dw.txt"; [ $rc -ne 0 ] && exit $rc
CMD="tools/dw_bench.py --stages S1,S3 --iters 3" bash tools/pmc_run.sh "${1:-r5a}/pmc"
