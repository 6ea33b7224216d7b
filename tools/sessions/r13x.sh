#!/bin/bash
# round 6: the ResNet-50 B=32 bf16 step's design check against torch.autocast (printed distances) for DESIGN.md
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13x}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -s --timeout 500 --timeout-method thread tests/test_bs32_parity_gpu.py -k resnet50 > $O/design.log 2>&1
echo "exit $?"; grep -E "\[design\]|passed|failed" $O/design.log | cut -c1-400
