#!/bin/bash
# round 4: serial kernel trace of the classification step with the one-launch BatchNorms on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/${1:-r8d}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SV_BN_SMALL=1 SV_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/side0 -o run -- python3 $R/bench.py --workload classification --steps 3 --warmup 3 --no-cpu-baseline > $O/side0.json 2> $O/side0.err
rc=$?; echo "side0 rc=$rc"; exit $rc
