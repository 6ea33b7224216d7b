#!/bin/bash
# round 5: kernel stats of the eval forward (bench.py --inference), to rank its kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11x}
O=gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --inference --steps 5 --warmup 2 --no-cpu-baseline > "$ROOTDIR/$O/prof_bench.json" 2> "$ROOTDIR/$O/prof.err" || { tail -20 "$ROOTDIR/$O/prof.err"; exit 1; }
find "$ROOTDIR/$O/prof" -name "*kernel_trace.csv" -delete
cd "$ROOTDIR"
python tools/stats_md.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 7 "round 5 $N eval forward" "rocprofv3 --kernel-trace --stats -- python3 bench.py --inference --steps 5 --warmup 2 --no-cpu-baseline" 40 > $O/kernel_stats.md
head -40 $O/kernel_stats.md
