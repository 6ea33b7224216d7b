#!/bin/bash
# round 5: classification step eager vs graph-replayed (host-bound check), and the finish-launch bound in each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r11f}
mkdir -p $O
for r in 1 2; do
for v in "off none" "on none" "off bn_fin" "on bn_fin"; do
  set -- $v
  SV_BN_FOLD=0 SV_DIAG_SKIP=$([ $2 = none ] && echo "" || echo $2) timeout -k 10 300 python bench.py --workload classification --graph $1 --steps 30 --warmup 5 --no-cpu-baseline > $O/b_$1_$2_$r.json 2>>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_$1_$2_$r.json').read().strip().splitlines()[-1]); print('graph=$1 skip=$2', d['value'], d['ms_per_step'])"
done
done
