#!/bin/bash
# round 6 checkpoint on the current tree: the whole GPU suite, smoke(), the default bench line (with the CPU baseline
# leg, as the driver runs it), the classification line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOTDIR=$(pwd)
N=${1:-r13s}
O=$ROOTDIR/gpurun_out/$N
mkdir -p $O
timeout -k 10 900 python -u -m pytest --maxfail=8 -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
echo "suite exit $?"; grep -E "^FAILED|[0-9]+ passed|failed" $O/tests.log | tail -10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('train', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline'], d['main_queue']['busy_ms_per_step'])"
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_cls.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/bench_cls.json').read().strip().splitlines()[-1]); print('cls', d['value'], d['ms_per_step'])"
