#!/bin/bash
# round 5: kernel-trace budgets of the classification step (ResNet-50 256, bs32) and the ConvNeXt eval forward
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
N=${1:-r10m}
O=gpurun_out/$N
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof_cls -o run -- python3 bench.py --workload classification --steps 3 --warmup 2 --no-cpu-baseline > $O/cls.json 2> $O/cls.err || { tail -5 $O/cls.err; exit 1; }
python tools/stats_md.py $(find $O/prof_cls -name "*kernel_stats.csv" | head -1) 5 "round 5 $N classification" "rocprofv3 --kernel-trace --stats -- python3 bench.py --workload classification --steps 3 --warmup 2 --no-cpu-baseline" 40 > $O/cls_kernel_stats.md
head -45 $O/cls_kernel_stats.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof_inf -o run -- python3 bench.py --inference --steps 3 --warmup 2 --no-cpu-baseline > $O/inf.json 2> $O/inf.err || { tail -5 $O/inf.err; exit 1; }
python tools/stats_md.py $(find $O/prof_inf -name "*kernel_stats.csv" | head -1) 5 "round 5 $N eval forward" "rocprofv3 --kernel-trace --stats -- python3 bench.py --inference --steps 3 --warmup 2 --no-cpu-baseline" 40 > $O/inf_kernel_stats.md
head -30 $O/inf_kernel_stats.md
find $O -name "*kernel_trace.csv" -delete
