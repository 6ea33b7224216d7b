#!/bin/bash
# round 4: per-pass ResNet-50 @256 bs32 conv timings with rates (layer-1 narrow convs vs the rest)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9m}
mkdir -p $O
timeout -k 10 300 python tools/conv_bench.py --iters 20 > $O/conv.txt 2>&1
rc=$?; cat $O/conv.txt; exit $rc
