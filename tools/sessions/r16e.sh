#!/bin/bash
# round 6 (re-entry): the pinned cross-lane fused-MLP-backward build's run-to-run test (tests/test_mlp_xlane_gpu.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r16e}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mlp_xlane_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -3 $O/t.txt
