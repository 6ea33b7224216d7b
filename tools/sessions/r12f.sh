#!/bin/bash
# round 5 final tree (after the cross-lane butterflies and the eval one-pass depthwise + LayerNorm): full GPU suite,
# smoke(), the default bench line, classification and eval forward lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r12f}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/cls.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/cls.json').read().strip().splitlines()[-1]); print('cls', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --inference --steps 20 --warmup 5 --no-cpu-baseline > $O/inf.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]); print('inf', d['value'], d['ms_per_step'])"
