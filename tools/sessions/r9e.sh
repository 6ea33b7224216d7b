#!/bin/bash
# round 4: production-schedule GEMM parity incl. ConvNeXt-large bs64 shapes; base/large bench after the split change
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9e}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gemm_family_gpu.py -k "production" > $O/tests.log 2>&1
rc=$?; grep "\[bs32\]\|passed\|failed" $O/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --backbone convnext_large --batch 64 --steps 5 --warmup 2 --no-cpu-baseline > $O/large.json 2>>$O/bench.err || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/base.json 2>>$O/bench.err || exit $?
for f in large base; do python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
