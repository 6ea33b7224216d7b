#!/bin/bash
# round 4: ResNet-50 classification serial kernel budget (side stream off) and the conv passes' GPU-side
# durations (kernel trace of tools/conv_bench.py: the event timing there includes host launch gaps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/${1:-r8a}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SV_SIDE_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/side0 -o run -- python3 $R/bench.py --workload classification --steps 3 --warmup 3 --no-cpu-baseline > $O/side0.json 2> $O/side0.err
rc=$?; echo "side0 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/side1 -o run -- python3 $R/bench.py --workload classification --steps 3 --warmup 3 --no-cpu-baseline > $O/side1.json 2> $O/side1.err
rc=$?; echo "side1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/conv -o run -- python3 $R/tools/conv_bench.py --iters 10 > $O/conv_bench.txt 2>&1
rc=$?; echo "conv rc=$rc"; exit $rc
