#!/bin/bash
# round 5: AdamW variant (2 groups per lane per round, non-temporal stores) -- standalone timing, tests, step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11p}
mkdir -p $O
for v in 0 1 0 1; do SV_ADAMW_V2=$v timeout -k 10 120 python tools/adamw_bench.py 2>/dev/null | tail -1 || exit 1; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_kernels_gpu.py::test_adamw_and_clip" tests/test_trainer_gpu.py tests/test_golden_r2_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
for v in 0 1; do
  SV_ADAMW_V2=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_${r}.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_${r}.json').read().strip().splitlines()[-1]); print('adamw_v2=$v', d['value'], d['ms_per_step'])"
done
done
