#!/bin/bash
# round 4: kernel trace of the ConvNeXt-base eval forward (bench.py --inference)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$R/gpurun_out/${1:-r9o}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --inference --steps 10 --warmup 3 --no-cpu-baseline > $O/inf.json 2> $O/inf.err || exit $?
tail -1 $O/inf.json
