#!/bin/bash
# round 6: classification (ResNet-50 bs32) step trace -- queue breakdown and main-queue gaps (host-paced or GPU-bound?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13w}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 5 --warmup 3 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 25 > $O/queues.txt && head -45 $O/queues.txt
python tools/queue_gaps.py $KT 10 > $O/gaps.txt; tail -16 $O/gaps.txt
gzip -f $KT
timeout -k 10 300 python tools/host_profile_resnet.py > $O/host_time.txt 2>&1 || true
tail -8 $O/host_time.txt
