#!/bin/bash
# round 5: classification step trace -- per-queue breakdown (tools/queue_breakdown.py) and the origin of the
# runtime's blit kernels (tools/copy_origin.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11b}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
HT=$(find $O/prof -name "*hip_api_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 25 > $O/queues.txt && cat $O/queues.txt
python tools/copy_origin.py $KT $HT > $O/copies.txt && cat $O/copies.txt
gzip -f $KT; rm -f $HT
