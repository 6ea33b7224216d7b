#!/bin/bash
# round 3 checkpoint: the full -m gpu suite and smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r4g}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $OUT/tests.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" "$OUT/tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $OUT/smoke.txt)"
exit $rc
