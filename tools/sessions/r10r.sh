#!/bin/bash
# round 5 measurement set on the fused-MLP forward + backward tree: full GPU suite, default bench (CPU baseline in the run), classification
# and eval lines, rocprof kernel stats, PMC traffic / MFMA passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
N=${1:-r10r}
bash tools/gpu_measure.sh $N || exit 1
timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$N/bench_inf.json 2>/dev/null || exit 1
CLOCK=0 bash tools/gpu_pmc.sh $N/pmc || exit 1
python tools/stats_md.py $(find gpurun_out/$N/prof -name "*kernel_stats.csv" | head -1) 5 "round 5 $N" "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline" 40 > gpurun_out/$N/kernel_stats.md
head -20 gpurun_out/$N/kernel_stats.md
