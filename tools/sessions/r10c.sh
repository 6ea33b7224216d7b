#!/bin/bash
# round 5: fused MLP standalone timing + a kernel-trace profile of the bench step with the fused MLP
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r10c}
mkdir -p $O
timeout -k 10 300 python tools/mlp_bench.py --shapes base-S1,base-S2,large-S1,base-S3 > $O/mlp_bench.txt 2>&1 || { tail -20 $O/mlp_bench.txt; exit 1; }
cat $O/mlp_bench.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
python tools/stats_md.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 5 "r10c fused MLP" "rocprofv3 --kernel-trace --stats bench.py --steps 3 --warmup 2" 40 > $O/kernel_stats.md
head -30 $O/kernel_stats.md
