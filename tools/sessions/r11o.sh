#!/bin/bash
# round 5: head-loss kernel (wave-reduction) tests + classification line; ConvNeXt eval-forward kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11o}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_head_loss_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/b_cls.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/b_cls.json').read().strip().splitlines()[-1]); print('cls', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_inf" -o run -- python3 "$ROOTDIR/bench.py" --inference --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_inf.json" 2> "$O/prof_inf.err" || { tail -5 "$O/prof_inf.err"; exit 1; }
find "$O/prof_inf" -name "*kernel_trace.csv" -delete
cd "$ROOTDIR"
python tools/stats_md.py $(find $O/prof_inf -name "*kernel_stats.csv" | head -1) 7 "round 5 $N eval forward" "rocprofv3 --kernel-trace --stats -- python3 bench.py --inference --steps 5 --warmup 2 --no-cpu-baseline" 30 > $O/inf_kernel_stats.md
head -30 $O/inf_kernel_stats.md
