#!/bin/bash
# round 6: kernel trace of the current default training step -- per-queue breakdown and the main queue's idle gaps
# (what the critical path waits for)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13n}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 30 > $O/queues.txt && head -50 $O/queues.txt
python tools/queue_gaps.py $KT 15 > $O/gaps.txt; tail -40 $O/gaps.txt
ST=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/stats_md.py $ST 5 "round 6 $N" "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline" 40 > $O/kernel_stats.md
gzip -f $KT
