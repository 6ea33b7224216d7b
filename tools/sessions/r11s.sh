#!/bin/bash
# round 5: the last block's fc1 / depthwise wgrads on the main stream BEFORE the stem backward (SV_TAIL_MAIN=2) --
# schedule-knob bitwise test, step A/B against the default, full GPU suite first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11s}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for v in 0 2; do
  SV_TAIL_MAIN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('tail=$v', d['value'], d['ms_per_step'])"
done
done
