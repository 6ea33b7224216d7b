#!/bin/bash
# round 4: cap on the main stream's backward GEMM grids (SV_MAIN_BWD_CAP): how much the static persistent tile
# lists lose when the side stream's wgrad holds half the chip at launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r9u}
mkdir -p $O
for i in 1 2; do
  for v in 0 128 192 224; do
    SV_MAIN_BWD_CAP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${v}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('cap=$v', d['value'], d['ms_per_step'])"
  done
done
