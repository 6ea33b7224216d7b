#!/bin/bash
# round 5: ConvNeXt-base bs32 training step trace -- per-queue breakdown (main / side stream busy time by kernel family)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r12a}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 30 > $O/queues.txt && head -70 $O/queues.txt
gzip -f $KT
