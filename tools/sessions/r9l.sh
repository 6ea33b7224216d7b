#!/bin/bash
# round 4: the side stream's weight-gradient GEMM family in-step (SV_WGRAD_IMPL 0 = v9 dispatch, 2 = v2, 3 = v3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9l}
mkdir -p $O
for i in 1 2 3; do
  for v in 0 2 3; do
    SV_WGRAD_IMPL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('impl=$v', d['value'], d['ms_per_step'])"
  done
done
