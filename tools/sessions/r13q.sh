#!/bin/bash
# round 6: the step on a high-priority stream (SV_MAIN_STREAM_PRIO=1) against the default, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13q}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
for f in 1 0 1 0; do
  SV_MAIN_STREAM_PRIO=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$f.json 2> $O/bench_$f.err || { tail -5 $O/bench_$f.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('main_prio=$f train', d['value'], d['ms_per_step'], d['main_queue']['busy_ms_per_step'])"
done
SV_MAIN_STREAM_PRIO=1 timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls_1.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/bench_cls_1.json').read().strip().splitlines()[-1]); print('main_prio=1 cls', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls_0.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/bench_cls_0.json').read().strip().splitlines()[-1]); print('main_prio=0 cls', d['value'], d['ms_per_step'])"
