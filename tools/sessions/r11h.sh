#!/bin/bash
# round 5: chunk-split BatchNorm finishes A/B (interleaved, 3 rounds) + kernel trace of the split form
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r11h}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
for r in 1 2 3; do
for v in 0 1; do
  SV_FIN_SPLIT=$v timeout -k 10 300 python bench.py --workload classification --steps 40 --warmup 8 --no-cpu-baseline > $O/b_split${v}_$r.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_split${v}_$r.json').read().strip().splitlines()[-1]); print('split=$v', d['value'], d['ms_per_step'])"
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 "$ROOTDIR/bench.py" --workload classification --steps 3 --warmup 2 --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof.err" || { tail -20 "$O/prof.err"; exit 1; }
cd "$ROOTDIR"
KT=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/queue_breakdown.py $KT 25 > $O/queues.txt && head -40 $O/queues.txt
gzip -f $KT
