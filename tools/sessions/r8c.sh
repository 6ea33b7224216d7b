#!/bin/bash
# round 4: classification A/B, one-launch BatchNorms on / off, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r8c}
mkdir -p $O
for i in 1 2 3; do
  for s in 1 0; do
    SV_BN_SMALL=$s timeout -k 10 300 python bench.py --workload classification --steps 50 --warmup 10 --no-cpu-baseline > $O/cls_small${s}_$i.json 2>>$O/bench.err || exit $?
    python -c "import json; d=json.loads(open('$O/cls_small${s}_$i.json').read().strip().splitlines()[-1]); print('small $s', d['value'], d['ms_per_step'])"
  done
done
