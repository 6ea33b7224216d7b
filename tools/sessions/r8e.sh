#!/bin/bash
# round 4: ResNet-50 3x3 conv passes at forced split-K depths (GPU-side durations from a kernel trace)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/${1:-r8e}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for sp in 1 2 4 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/s$sp -o run -- python3 $R/tools/conv_bench.py --iters 10 --only 3x3 --split $sp > $O/s$sp.txt 2>&1
  rc=$?; echo "split $sp rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
