#!/bin/bash
# round 4: the fold passes standalone (tools/fold_bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9zf}
mkdir -p $O
timeout -k 10 300 python tools/fold_bench.py > $O/fold.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/fold.txt; exit $rc
