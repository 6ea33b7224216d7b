#!/bin/bash
# round 4: reduction kernels after the ragged-n fix, then the rest of the GPU suite from where r8i stopped
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8l}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; grep -E "^FAILED" $O/tests.log | head -20; exit $rc
