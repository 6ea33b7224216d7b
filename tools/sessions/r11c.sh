#!/bin/bash
# round 5: upper bounds for the ResNet BatchNorm launches -- classification bench with the fold (finish) launches
# or the forward activation launches skipped (SV_DIAG_SKIP; results garbage, timing only), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11c}
mkdir -p $O
for r in 1 2; do
for v in none bn_fin bn_act bn_fin,bn_act; do
  SV_DIAG_SKIP=$([ $v = none ] && echo "" || echo $v) timeout -k 10 300 python bench.py --workload classification --steps 30 --warmup 5 --no-cpu-baseline > $O/b_${v}_$r.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
done
