#!/bin/bash
# round 5 measurement set (ResNet bf16 gradient stream, split BatchNorm folds, fused classification loss): full GPU
# suite, default bench (CPU baseline in the run), classification line (30 steps) + its kernel trace and queue
# breakdown, eval line, rocprof kernel stats, PMC traffic / MFMA passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11n}
O=$ROOTDIR/gpurun_out/$N
bash tools/gpu_measure.sh $N || exit 1
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls30.json 2>/dev/null || exit 1
head -c 200 $O/bench_cls30.json; echo
timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_inf.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/cls_trace" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline > "$O/cls_trace_bench.json" 2> "$O/cls_trace.err" || exit 1
cd "$ROOTDIR"
KT=$(find $O/cls_trace -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 25 > $O/cls_queues.txt && head -3 $O/cls_queues.txt
gzip -f $KT
CLOCK=0 bash tools/gpu_pmc.sh $N/pmc || exit 1
python tools/stats_md.py $(find gpurun_out/$N/prof -name "*kernel_stats.csv" | head -1) 5 "round 5 $N" "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline" 40 > gpurun_out/$N/kernel_stats.md
head -12 gpurun_out/$N/kernel_stats.md
